"""Parity of the exact chains bench.py times, at (or past) their workload sizes.

bench.py's legs run code paths the small parity tests never reach: the matrix-core exact-u8
+-16 motion search over many frame pairs feeding the SRC_INTER residual DCT + quantiser (cfg4,
in one piece and pipelined over chunks of pairs), the fused intra kernel writing a batch whose
output lies past 4 GiB (cfg3), and the chunked cfg5 step with its side-stream histograms.
These tests run those chains on the bench's own synthetic generators and compare sampled
frames (whole frames, every block) with the C/NumPy oracle (oracle.c_inter_encode:
motion.py:8-97 + videocodec.py:52-73 + dct.py:12-28 + patchquant.py:44-60)."""
import numpy as np
import pytest

from oracle import c_inter_encode
from oracle import ivc_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import bench  # noqa: E402  (the bench's own synthetic generators)
import ivclab_amd.device as D  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402

TABLE = PatchQuant(1.0).get_quantization_table()


def assert_bits(a, b, what=""):
    a, b = np.asarray(a), np.asarray(b)
    assert a.dtype == b.dtype, f"{what}: dtype {a.dtype} != {b.dtype}"
    assert a.shape == b.shape, f"{what}: shape {a.shape} != {b.shape}"
    if a.tobytes() != b.tobytes():
        bad = np.flatnonzero(a.reshape(-1) != b.reshape(-1))
        raise AssertionError(f"{what}: {bad.size} differing elements, first at {bad[0]}")


@pytest.mark.parametrize("chunks", [0, 3])
def test_inter_encode_sr16_1080p_across_s2_chunks(tune, chunks):
    """cfg4's chain at its frame size: 40 frames of the bench's 1080p sequence at sr = 16
    (me_mfma16x2_kernel then the residual encoder), in one piece and pipelined over 3 chunks of
    pairs (the inter_chunks override: the search of chunk j + 1 beside the residual encode of
    chunk j on the second stream).  Pairs 0, 31, 32 and 38 are checked whole — every motion
    vector and every quantised residual coefficient — against the C oracle chain."""
    tune("inter_chunks", chunks)
    dev = torch.device("cuda:0")
    F, H, W, sr = 40, 1080, 1920, 16
    seq = bench.inter_frames(F, H, W, seed=4, dev=dev)
    mv = torch.full((F - 1, H // 8, W // 8), -1, dtype=torch.int64, device=dev)
    q = torch.full((F - 1, H // 8, W // 8, 3, 64), -7, dtype=torch.int32, device=dev)
    D.inter_encode(seq, sr, TABLE, mv, q)
    torch.cuda.synchronize()
    host = seq.cpu().numpy()
    for p in (0, 31, 32, F - 2):
        wmv, wq = c_inter_encode(host[p], host[p + 1], sr, 1.0)
        assert_bits(mv[p].cpu().numpy(), wmv[..., 0], f"mv pair {p}")
        assert_bits(q[p].cpu().numpy(), wq.reshape(H // 8, W // 8, 3, 64), f"q pair {p}")
    # every pair was written (no chunk skipped): indices in range, no sentinel left
    m = mv.cpu().numpy()
    assert m.min() >= 0 and m.max() < (2 * sr + 1) ** 2


def test_inter_encode_sr16_8k_chunks():
    """cfg5's chain at its own frame size (BASELINE configs[4], 7680x4320): 4 frames of the
    bench's cfg5 sequence (3 pairs): mv and q of the top, middle and bottom
    block-row stripes of every pair against the C oracle chain (motion.py:8-58,
    patchquant.py:44-60); every pair written; and the chunked side-stream histograms of the
    cfg5 step (1 pair per chunk) equal one call followed by main-stream histograms."""
    import ivclab_amd._native as N
    dev = torch.device("cuda:0")
    F, H, W, sr = 4, 4320, 7680, 16
    seq = bench.inter_frames(F, H, W, seed=5, dev=dev)
    P, h = F - 1, H // 8
    nmv = (2 * sr + 1) ** 2
    mv = torch.full((P, h, W // 8), -1, dtype=torch.int64, device=dev)
    q = torch.full((P, h, W // 8, 3, 64), -7, dtype=torch.int32, device=dev)
    D.inter_encode(seq, sr, TABLE, mv, q)
    hist1 = torch.zeros(bench.HIST_BINS + nmv, dtype=torch.int64, device=dev)
    D.histogram(q.view(-1), bench.HIST_LO, hist1[:bench.HIST_BINS])
    D.histogram(mv.view(-1), 0, hist1[bench.HIST_BINS:])
    torch.cuda.synchronize()
    host = seq.cpu().numpy()
    for p in range(P):
        for rows in ((0, 3), (h // 2 - 1, h // 2 + 2), (h - 3, h)):
            wmv, wq = c_inter_encode(host[p], host[p + 1], sr, 1.0, rows=rows)
            assert_bits(mv[p, rows[0]:rows[1]].cpu().numpy(), wmv[..., 0], f"mv pair {p} rows {rows}")
            assert_bits(q[p, rows[0]:rows[1]].cpu().numpy(),
                        wq.reshape(rows[1] - rows[0], W // 8, 3, 64), f"q pair {p} rows {rows}")
    m = mv.cpu().numpy()
    assert m.min() >= 0 and m.max() < nmv
    assert int((q == -7).all(dim=-1).sum().item()) == 0   # no block left unwritten
    # the cfg5 step itself (bench.make_sharded_step): 1 pair per chunk, side-stream histograms
    mv2, q2 = torch.empty_like(mv), torch.empty_like(q)
    hist2 = torch.zeros_like(hist1)
    step = bench.make_sharded_step(D, N, seq, P, sr, TABLE, mv2, q2, hist2, 1, 2, False,
                                   torch.cuda.Stream(device=dev))
    step()
    torch.cuda.synchronize()
    assert torch.equal(mv2, mv) and torch.equal(q2, q)
    assert_bits(hist2.cpu().numpy(), hist1.cpu().numpy(), "chunked side-stream histograms")
    assert int(hist1[:bench.HIST_BINS].sum().item()) == q.numel()


def test_inter_encode_sr16_zigzag_and_motion_range():
    """The zig-zag variant of the same chain on a sequence whose motion spans the whole
    +-16 window (large shifts, flat and textured regions), 4 pairs checked whole."""
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(416)
    H, W, sr = 272, 480, 16
    lo = rng.integers(0, 256, (H // 4 + 12, W // 4 + 12)).astype(np.float64)
    base = np.kron(lo, np.ones((4, 4))) + rng.integers(-3, 4, (H + 48, W + 48))
    base = np.clip(base, 0, 255).astype(np.uint8)
    shifts = [(0, 0), (16, -16), (-16, 16), (7, -13), (0, 0)]
    frames = np.stack([base[24 + dy:24 + dy + H, 24 + dx:24 + dx + W] for dy, dx in shifts])
    frames[2, 40:120, 100:300] = 90                               # flat: tie-break path
    F = len(frames)
    seq = torch.from_numpy(np.ascontiguousarray(frames)).to(dev)
    mv = torch.empty((F - 1, H // 8, W // 8), dtype=torch.int64, device=dev)
    q = torch.empty((F - 1, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    D.inter_encode(seq, sr, TABLE, mv, q, zigzag=True)
    torch.cuda.synchronize()
    for p in range(F - 1):
        wmv, wq = c_inter_encode(frames[p], frames[p + 1], sr, 1.0, zigzag=True)
        assert_bits(mv[p].cpu().numpy(), wmv[..., 0], f"mv pair {p}")
        assert_bits(q[p].cpu().numpy(), wq, f"q pair {p}")


def test_intra_encode_batch_past_4gib():
    """cfg3's kernel on 48 4K frames of the bench generator: the int32 output is 4.78 GB, so
    the buffer-descriptor rebase has to carry offsets past 4 GiB.  Frames 0, 23, 24 and 47
    (first, either side of the middle, last: the last lies entirely beyond 4 GiB) are checked
    whole against the oracle; the rest are checked to have been written."""
    dev = torch.device("cuda:0")
    F, H, W = 48, 2160, 3840
    frames = bench.intra_frames(F, H, W, seed=3, dev=dev).view(F, H, W, 1)
    out = torch.full((F, H // 8, W // 8, 3, 64), -(1 << 30), dtype=torch.int32, device=dev)
    assert out.numel() * 4 > (1 << 32) + H // 8 * W // 8 * 3 * 64 * 4
    D.intra_encode(frames, TABLE, out)
    torch.cuda.synchronize()
    for f in (0, 23, 24, F - 1):
        want = O.intra_encode(frames[f].cpu().numpy(), 1.0).reshape(H // 8, W // 8, 3, 64)
        assert_bits(out[f].cpu().numpy(), want, f"frame {f}")
    # the sentinel is outside every quantised value's range: nothing left unwritten
    assert int((out == -(1 << 30)).sum().item()) == 0


def test_decode_batch_48_4k_frames():
    """The decode chain at workload size (IntraCodec.symbols2image, intracodec.py:84-146):
    48 4K frames encoded by the fused intra kernel with zig-zag ([48, 270, 480, 3, 64] int32,
    4.78 GB), then (a) ivc_intra_decode_image of the coefficients and (b) the full device chain
    from the frames' zero-run symbol stream (ivc_symbols2image_dev: zero-run decode ->
    un-zig-zag -> dequantise -> IDCT -> unpatch -> ycbcr2rgb) into [48, 2160, 3840, 3] float64
    (9.6 GB).  Frames 0, 23, 24, 47 are checked whole against the oracle (O.intra_decode,
    unpatch, ycbcr2rgb)."""
    dev = torch.device("cuda:0")
    F, H, W = 48, 2160, 3840
    frames = bench.intra_frames(F, H, W, seed=3, dev=dev).view(F, H, W, 1)
    q = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    D.intra_encode(frames, TABLE, q, zigzag=True)
    out = torch.full((F, H, W, 3), float("nan"), dtype=torch.float64, device=dev)
    D.intra_decode_image(q, TABLE, out, unzigzag=True, to_rgb=False)
    torch.cuda.synchronize()
    picks = (0, 23, 24, F - 1)
    for f in picks:
        want = O.unpatch(O.intra_decode(q[f].cpu().numpy(), 1.0, unzigzag=True))
        assert_bits(out[f].cpu().numpy(), want, f"decoded frame {f}")
    # (b) from the symbol stream, RGB
    nblk = q.numel() // 64
    offs = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
    probe = torch.empty(1, dtype=torch.int32, device=dev)
    D.zerorun_encode(q.view(nblk, 64), offs, probe)
    sym = torch.empty(int(offs[-1].item()), dtype=torch.int32, device=dev)
    D.zerorun_encode(q.view(nblk, 64), offs, sym)
    del q, offs
    err = torch.full((3,), -1, dtype=torch.int64, device=dev)
    out.fill_(float("nan"))
    D.symbols2image(sym, 3, TABLE, out, err, to_rgb=True)
    torch.cuda.synchronize()
    assert err.tolist() == [0, 0, 0]
    for f in picks:
        qf = O.intra_encode(frames[f].cpu().numpy(), 1.0, zigzag=True)
        want = O.ycbcr2rgb(O.unpatch(O.intra_decode(qf, 1.0, unzigzag=True)))
        assert_bits(out[f].cpu().numpy(), want, f"symbols2image frame {f}")


def test_chunked_inter_encode_with_side_stream_histograms():
    """The cfg5 step shape: inter_encode in chunks of 2 pairs with each chunk's coefficient
    and motion-vector histograms on a side stream while the next chunk is encoded, at reduced
    histogram occupancy, gives the same mv, q and histograms as one call followed by the
    histograms on the main stream; and with the coefficients' histogram accumulated by the
    encoder itself (inter_encode(hist=...), the bench's form) the histogram is the same."""
    import ivclab_amd._native as N
    dev = torch.device("cuda:0")
    F, H, W, sr = 7, 1080, 1920, 16
    seq = bench.inter_frames(F, H, W, seed=5, dev=dev)
    P = F - 1
    nmv = (2 * sr + 1) ** 2

    def run(chunk, wg, enc_hist=False):
        mv = torch.empty((P, H // 8, W // 8), dtype=torch.int64, device=dev)
        q = torch.empty((P, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
        hist = torch.zeros(bench.HIST_BINS + nmv, dtype=torch.int64, device=dev)
        main, side = torch.cuda.current_stream(), torch.cuda.Stream(device=dev)
        L = N.lib()
        prev = L.ivc_histogram_occupancy()
        N.check(L.ivc_set_histogram_occupancy(wg))
        try:
            for p0 in range(0, P, chunk):
                p1 = min(p0 + chunk, P)
                if enc_hist:
                    D.inter_encode(seq[p0:p1 + 1], sr, TABLE, mv[p0:p1], q[p0:p1], stream=main,
                                   hist=hist[:bench.HIST_BINS], hist_lo=bench.HIST_LO)
                else:
                    D.inter_encode(seq[p0:p1 + 1], sr, TABLE, mv[p0:p1], q[p0:p1], stream=main)
                side.wait_stream(main)
                if not enc_hist:
                    D.histogram(q[p0:p1].view(-1), bench.HIST_LO, hist[:bench.HIST_BINS], stream=side)
                D.histogram(mv[p0:p1].view(-1), 0, hist[bench.HIST_BINS:], stream=side)
            main.wait_stream(side)
            torch.cuda.synchronize()
        finally:
            N.check(L.ivc_set_histogram_occupancy(prev))
        return mv.cpu().numpy(), q.cpu().numpy(), hist.cpu().numpy()

    mv1, q1, h1 = run(P, 0)
    mv2, q2, h2 = run(2, 2)
    mv3, q3, h3 = run(2, 2, enc_hist=True)
    assert_bits(mv2, mv1, "mv chunked")
    assert_bits(q2, q1, "q chunked")
    assert_bits(h2, h1, "hist chunked")
    assert_bits(q3, q1, "q chunked, encoder histogram")
    assert_bits(h3, h1, "hist chunked, encoder histogram")
    assert h1[:bench.HIST_BINS].sum() == q1.size and h1[bench.HIST_BINS:].sum() == mv1.size
    assert np.array_equal(h1[bench.HIST_BINS:], O.histogram(mv1, 0, nmv))
    assert np.array_equal(h1[:bench.HIST_BINS], O.histogram(q1, bench.HIST_LO, bench.HIST_BINS))
    # and pair 3 of the chunked run against the oracle
    host = seq.cpu().numpy()
    wmv, wq = c_inter_encode(host[3], host[4], sr, 1.0)
    assert_bits(mv2[3], wmv[..., 0], "mv pair 3")
    assert_bits(q2[3], wq.reshape(H // 8, W // 8, 3, 64), "q pair 3")


def test_me_matrix_core_search_repeatable():
    """The +-16 matrix-core search relaunched many times over 16 8K pairs (the persistent grid
    walks ~15 tiles per workgroup, so every workgroup crosses its loop-header barrier many
    times) gives the same vectors every time: before every barrier drained its LDS writes
    (ivc_internal.h lds_barrier) the cross-wave merge read a stale per-wave entry in ~4 % of
    cfg5 steps (profiles/r05ai_race_probe.log).  A guard, not a proof: a rare race can pass."""
    dev = torch.device("cuda:0")
    F, H, W, sr = 17, 4320, 7680, 16
    seq = bench.inter_frames(F, H, W, seed=5, dev=dev)
    mv = torch.empty((F - 1, H // 8, W // 8), dtype=torch.int64, device=dev)
    D.motion_estimate(seq[:-1], seq[1:], sr, mv, exact_u8=True)
    ref = mv.clone()
    differ = 0
    for _ in range(60):
        mv.fill_(-1)
        D.motion_estimate(seq[:-1], seq[1:], sr, mv, exact_u8=True)
        differ += not torch.equal(mv, ref)
    assert differ == 0, f"{differ} of 60 relaunches gave different motion vectors"
    # and one block-row stripe of pair 0 against the C oracle
    host = seq[:2].cpu().numpy()
    wmv, _ = c_inter_encode(host[0], host[1], sr, 1.0, rows=(0, 3))
    assert_bits(ref[0, 0:3].cpu().numpy(), wmv[..., 0], "mv pair 0 rows 0-2")


@pytest.mark.parametrize("C,chunks", [(3, None), (1, None), (3, 3), (1, 16)])
def test_symbols2image_fused_adversarial(tune, C, chunks):
    """The fused symbols -> image kernel (ivc_decode.hip sym_image_kernel: zero-run expansion
    into LDS, dequantise, IDCT, unpatch, ycbcr2rgb; intracodec.py:84-146 + zerorun.py:44-88)
    alone — the s2i_no_fallback override keeps the general decoder from overwriting its image — on
    coefficients built to stress it: all-zero blocks (one EOB per block-plane, so 4096-symbol
    tiles hold dozens of group starts), densest blocks (value, 0, run 1, ... = 97 symbols per
    block-plane), long runs, a value at zig-zag position 63, large DCs, a ragged last group
    (w = 125 block columns) and a stream of 130k-380k symbols over 30-90 tiles; against the
    oracle chain (ZeroRunCoder.decode, unflatten, dequantise, IDCT, unpatch, ycbcr2rgb)."""
    tune("s2i_no_fallback", 1)
    if chunks:     # the pipelined call (ivc_entropy.hip s2i_pipelined) on a stream of 30-90 tiles
        tune("s2i_chunks", chunks)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(40 + C)
    F, H, W = 2, 128, 1000
    h, w = H // 8, W // 8
    q = rng.integers(-3, 4, (F, h, w, C, 64)).astype(np.int32)
    q[..., 8:] *= rng.random(q[..., 8:].shape) < 0.15
    kind = rng.integers(0, 5, (F, h, w, C))
    q[kind == 0] = 0                                              # all-zero block-planes
    dense = np.where(np.arange(64) % 2 == 1, 5, 0).astype(np.int32)
    q[kind == 1] = dense                                          # (0, 1, 5) x 32 + EOB = 97
    q[kind == 2, 1:63] = 0                                        # one long run, then pos 63
    q[kind == 2, 63] = -7
    q[..., 0] = np.where(kind == 3, rng.integers(-1500, 1500, kind.shape), q[..., 0])
    sym = np.asarray(O.zerorun_encode_fast(q.reshape(-1, 64)), dtype=np.int32)
    assert sym.size > 120_000
    table = PatchQuant(0.8).get_quantization_table()
    out = torch.full((F, H, W, 3), float("nan"), dtype=torch.float64, device=dev)
    err = torch.full((3,), -1, dtype=torch.int64, device=dev)
    D.symbols2image(torch.from_numpy(sym).to(dev), C, table, out, err, to_rgb=(C == 3))
    torch.cuda.synchronize()
    assert err.tolist() == [0, 0, 0]
    for f in range(F):
        want = O.unpatch(O.intra_decode(q[f], 0.8, unzigzag=True))
        if C == 3:
            want = O.ycbcr2rgb(want)
        assert_bits(out[f].cpu().numpy(), want, f"fused symbols2image C={C} frame {f}")


@pytest.mark.parametrize("chunks", [1, 4, 13])
def test_symbols2image_pipelined_rejects_and_falls_back(tune, chunks):
    """A malformed block (a run past 64 coefficients) in the middle of a 40-tile stream: the
    fused path — one pass or pipelined over chunks of tiles — rejects the stream
    (the s2i_no_fallback override reports err[0] = -100), and with the fallback the call reports the
    reference's error, as ZeroRunCoder.decode raises it (zerorun.py:66-70)."""
    from ivclab_amd.image import IntraCodec
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(77)
    F, H, W, C = 1, 128, 1000, 3
    q = rng.integers(-3, 4, (F, H // 8, W // 8, C, 64)).astype(np.int32)
    q[..., 8:] *= rng.random(q[..., 8:].shape) < 0.15
    sym = np.asarray(O.zerorun_encode_fast(q.reshape(-1, 64)), dtype=np.int32)
    eobs = np.flatnonzero(sym == 4000)
    cut = eobs[len(eobs) // 2] + 1                     # a block boundary mid-stream
    bad = np.concatenate([sym[:cut], [0, 70], sym[cut:]]).astype(np.int32)
    table = PatchQuant(1.0).get_quantization_table()
    tune("s2i_chunks", chunks)
    out = torch.empty((F, H, W, 3), dtype=torch.float64, device=dev)
    err = torch.full((3,), -1, dtype=torch.int64, device=dev)
    # the clean stream decodes identically whatever the chunking
    D.symbols2image(torch.from_numpy(sym).to(dev), C, table, out, err, to_rgb=True)
    torch.cuda.synchronize()
    assert err.tolist() == [0, 0, 0]
    want0 = O.ycbcr2rgb(O.unpatch(O.intra_decode(q[0], 1.0, unzigzag=True)))
    assert_bits(out[0].cpu().numpy(), want0, f"clean stream, chunks={chunks}")
    tune("s2i_no_fallback", 1)
    D.symbols2image(torch.from_numpy(bad).to(dev), C, table, out, err, to_rgb=True)
    torch.cuda.synchronize()
    assert int(err[0]) == -100, err.tolist()
    tune("s2i_no_fallback", 0)
    codec = IntraCodec(quantization_scale=1.0)
    with pytest.raises(Exception) as got:
        codec.symbols2image(bad, (H, W, 3))
    with pytest.raises(Exception) as want:
        O.zerorun_decode(list(bad), (H // 8, W // 8, C))
    assert type(got.value) is type(want.value) and str(got.value) == str(want.value)
