"""Parity of the HIP path (through the C-ABI, via the ivclab-signature classes) with the
oracle and with the reference's golden vectors.  Bar: bit-exact for every output (float
DCT outputs included — the kernels reproduce pocketfft's op order exactly, which is
stricter than the 1e-5 relative tolerance north_star allows for float DCT)."""
import numpy as np
import pytest

from oracle import c_motion_compensate, c_motion_vectors
from oracle import ivc_oracle as O

pytestmark = pytest.mark.gpu

IA = pytest.importorskip("ivclab_amd")
from ivclab_amd import MotionCompensator, Patcher, PatchQuant, ZigZag  # noqa: E402
from ivclab_amd.signal import DiscreteCosineTransform  # noqa: E402
from ivclab_amd.signal.zigzag import zigzag_scan  # noqa: E402

DCT = DiscreteCosineTransform()
ALL_DTYPES = [np.uint8, np.int8, np.uint16, np.int16, np.uint32, np.int32, np.uint64,
              np.int64, np.float32, np.float64]


def bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def assert_bits(a, b, what=""):
    a, b = np.asarray(a), np.asarray(b)
    assert a.dtype == b.dtype, f"{what}: dtype {a.dtype} != {b.dtype}"
    assert a.shape == b.shape, f"{what}: shape {a.shape} != {b.shape}"
    if a.tobytes() != b.tobytes():
        bad = np.flatnonzero(a.reshape(-1).view(np.uint8) != b.reshape(-1).view(np.uint8))
        raise AssertionError(f"{what}: {bad.size} differing bytes, first at byte {bad[0]}")


def rand_array(rng, dtype, shape):
    dtype = np.dtype(dtype)
    if dtype.kind == "f":
        return (rng.normal(0, 80, shape)).astype(dtype)
    info = np.iinfo(dtype)
    lo, hi = max(info.min, -300), min(info.max, 300)
    return rng.integers(lo, hi + 1, shape).astype(dtype)


# ------------------------------------------------------------------------ DCT ----------
@pytest.mark.parametrize("C", [1, 3, 2])
@pytest.mark.parametrize("dtype", [np.uint8, np.float64, np.float32, np.int16])
def test_dct_of_patch_view_read_in_place(C, dtype):
    """DCT.transform(Patcher.patch(img)) reads the image in place (ivc_dct8x8_image: the
    kernel addresses the view, dct.py:12-28 on shape.py:45-54); the result equals the
    transform of the gathered view and the oracle's, for both directions, on a frame large
    enough for the chunked host pipeline and on one that is not."""
    rng = np.random.default_rng(7 + C)
    from ivclab_amd.signal.dct import patch_view_image
    for H, W in ((48, 72), (1080, 1920)):
        img = rand_array(rng, dtype, (H, W, C))
        p = Patcher().patch(img)
        assert patch_view_image(p) is not None
        for inv in (False, True):
            f = DCT.inverse_transform if inv else DCT.transform
            o = O.dct_inverse if inv else O.dct_transform
            got = f(p)
            assert_bits(got, f(np.ascontiguousarray(p)), f"view vs gathered C={C} {dtype} inv={inv}")
            if H == 48:
                assert_bits(got, o(p), f"view vs oracle C={C} {dtype} inv={inv}")
    # a view of a non-contiguous image is gathered as before
    img = rand_array(rng, dtype, (48, 72, C))[:, ::-1]
    p = Patcher().patch(img)
    assert patch_view_image(p) is None
    assert_bits(DCT.transform(p), O.dct_transform(p), "reversed view")


def test_host_pipeline_chunking_changes_nothing():
    """Host-buffer calls with page-locked results go in chunks on 3 streams
    (ivc_set_host_pipeline); every chunk size, and none, gives the same bits."""
    from ivclab_amd import _native as N
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (2160, 3840, 1), dtype=np.uint8)
    pq, zz, pt = PatchQuant(0.7), ZigZag(), Patcher()
    L = N.lib()
    outs = []
    prev = int(L.ivc_host_pipeline())
    assert prev == 0, "the library default runs host-buffer calls in one piece"
    try:
        for chunk in (0, 1 << 20, 3 << 20, 8 << 20):
            N.check(L.ivc_set_host_pipeline(chunk))
            d = DCT.transform(pt.patch(img))
            q = pq.quantize(d)
            z = zz.flatten(q)
            outs.append((d, q, z, pq.dequantize(q), zz.unflatten(z)))
    finally:
        N.check(L.ivc_set_host_pipeline(prev))
    assert int(L.ivc_host_pipeline()) == prev
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            assert_bits(a, b, "pipelined vs one piece")
    assert_bits(outs[0][2].reshape(-1, 64), O.zigzag_flatten(O.quantize(O.dct_transform(pt.patch(img)), 0.7)).reshape(-1, 64), "vs oracle")


def test_tiny_calls_zero_copy():
    """One (8, 8) block, a (3, 8, 8) stack, one zig-zag row: the tiny-call path (the kernel
    reads and writes a mapped page-locked block) against the oracle, many calls in a row."""
    rng = np.random.default_rng(5)
    pq = PatchQuant(0.5)
    zz = ZigZag()
    for _ in range(50):
        blk = rng.normal(0, 90, (8, 8))
        assert_bits(DCT.transform(blk), O.dct_transform(blk), "8x8")
        assert_bits(DCT.inverse_transform(blk), O.dct_inverse(blk), "8x8 inverse")
        stk = rng.normal(0, 40, (3, 8, 8))
        assert_bits(pq.quantize(stk), O.quantize(stk, 0.5), "3x8x8")
        q = pq.quantize(stk)
        assert_bits(pq.dequantize(q), O.dequantize(q, 0.5), "dequantize")
        z = zigzag_scan(blk.astype(np.int32))
        assert_bits(z, O.zigzag_scan(blk.astype(np.int32)), "zigzag_scan")


@pytest.mark.parametrize("server", [0, 1])
def test_tiny_server_and_launch_paths(server, tune):
    """The per-block calls through the resident tiny-call server (server 0, the default) and
    through one kernel launch each (server 1 = off): every DCT source dtype (float32 -> float32,
    the rest -> float64), forward and inverse, every norm; quantise and dequantise of (1, 8, 8)
    and (3, 8, 8) stacks of several dtypes in float64 and float32 arithmetic, the table changed
    between calls (the server's cached copy must follow); the server left idle long enough to
    exit and relaunched; a device-wide synchronisation right after a call (the resident wave
    leaves within its idle time)."""
    import time
    import torch
    tune("tiny_server", server)
    rng = np.random.default_rng(900 + server)
    for norm in ("ortho", "backward", "forward"):
        dct = DiscreteCosineTransform(norm=norm)
        for dt in (np.float64, np.float32, np.uint8, np.int16, np.int32, np.int64):
            x = (rng.normal(0, 60, (8, 8)) if dt in (np.float64, np.float32)
                 else rng.integers(0, 200, (8, 8))).astype(dt)
            assert_bits(dct.transform(x), O.dct_transform(x, norm=norm), f"dct {norm} {dt.__name__}")
            assert_bits(dct.inverse_transform(x), O.dct_inverse(x, norm=norm), f"idct {norm} {dt.__name__}")
    for scale in (1.0, 0.5, 0.15):
        pq = PatchQuant(scale)
        for C in (1, 3):
            for dt in (np.float64, np.float32, np.int16, np.int32):
                x = (rng.normal(0, 80, (C, 8, 8)) if dt in (np.float64, np.float32)
                     else rng.integers(-300, 300, (C, 8, 8))).astype(dt)
                assert_bits(pq.quantize(x), O.quantize(x, scale), f"quantize s={scale} C={C} {dt.__name__}")
                assert_bits(pq.dequantize(x.astype(np.int32)), O.dequantize(x.astype(np.int32), scale),
                            f"dequantize s={scale} C={C}")
    blk = rng.normal(0, 50, (8, 8))
    time.sleep(0.01)                                     # past the server's idle time: it leaves
    assert_bits(DCT.transform(blk), O.dct_transform(blk), "after idle exit")
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 0.1
    for _ in range(200):                                 # back to back
        blk = rng.normal(0, 50, (8, 8))
        assert_bits(DCT.transform(blk), O.dct_transform(blk), "loop")


def test_tiny_server_idle_exit_races():
    """Calls spaced around the server's 0.5 ms idle exit, so requests land just before, at and
    just after the resident wave leaves (the host must see it gone and relaunch, and the new
    wave must answer the pending request exactly once): every result against the oracle."""
    import time
    rng = np.random.default_rng(4242)
    pq = PatchQuant(0.75)
    for i in range(300):
        t_end = time.perf_counter() + rng.uniform(0.3e-3, 0.8e-3)
        while time.perf_counter() < t_end:
            pass
        if i % 2:
            b = rng.normal(0, 60, (8, 8))
            assert_bits(DCT.transform(b), O.dct_transform(b), f"dct after gap {i}")
        else:
            s = rng.normal(0, 40, (3, 8, 8))
            assert_bits(pq.quantize(s), O.quantize(s, 0.75), f"quantize after gap {i}")


@pytest.mark.parametrize("server", [0, 1])
def test_tiny_calls_from_threads(server, tune):
    """Per-block calls from 4 host threads at once (the C-ABI serialises a device's staged
    calls, so each thread's results must be its own): DCTs and quantisations of distinct data,
    each checked against the oracle, through the server and through the launch path."""
    import threading
    tune("tiny_server", server)
    errors = []

    def work(seed):
        try:
            rng = np.random.default_rng(seed)
            pq = PatchQuant(0.5 + 0.25 * (seed % 3))
            for _ in range(150):
                b = rng.normal(0, 60, (8, 8))
                np.testing.assert_array_equal(DCT.transform(b), O.dct_transform(b))
                s = rng.normal(0, 40, (3, 8, 8))
                np.testing.assert_array_equal(pq.quantize(s), O.quantize(s, pq.quantization_scale))
        except Exception as e:                           # noqa: BLE001 - reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=work, args=(1000 + i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:2]


def test_tiny_inline_capacity_mismatch():
    """Inputs of 513-1536 B through the tiny path (above the one-block DCT launcher's 512 B
    argument capacity, within the general one's): several blocks per DCT call, float64 stacks
    to quantise, int32 rows to zig-zag, interleaved with one-block calls so a stale page-locked
    block would show (with_tiny now stages an input it cannot inline)."""
    rng = np.random.default_rng(515)
    pq = PatchQuant(0.75)
    for i in range(20):
        one = rng.normal(0, 80, (8, 8))
        assert_bits(DCT.transform(one), O.dct_transform(one), "one block")
        for shape, dt in (((2, 8, 8), np.float64), ((3, 8, 8), np.float64), ((5, 8, 8), np.float32),
                          ((3, 8, 8), np.float32), ((24, 8, 8), np.uint8)):
            x = (rng.normal(0, 60, shape) if dt != np.uint8 else rng.integers(0, 256, shape)).astype(dt)
            assert 512 < x.nbytes <= 1536, x.nbytes
            assert_bits(DCT.transform(x), O.dct_transform(x), f"dct {shape} {dt.__name__}")
        stk = rng.normal(0, 40, (3, 8, 8))
        assert_bits(pq.quantize(stk), O.quantize(stk, 0.75), "quantize 1536 B")
        z = rng.integers(-50, 50, (4, 8, 8)).astype(np.int32)      # 1024 B
        assert_bits(zigzag_scan(z[i % 4]), O.zigzag_scan(z[i % 4]), "zigzag_scan")


def test_tiny_call_fast_paths_match_general_path():
    """The per-block fast paths of DCT.transform / PatchQuant.quantize / dequantize (small
    arrays straight to the C-ABI, cached table) give the general path's bits and the oracle's
    on what the reference's per-block loops pass (exercises/ch3/E3-1_claude.py:47-60: one
    channel of a patch view — non-contiguous float32 — then the (3, 8, 8) stack), read-only
    and byte-swapped inputs, C = 1 stacks that broadcast, and a table edited in place or a
    scale replaced between calls (the cache must notice)."""
    rng = np.random.default_rng(77)
    img = (rng.integers(0, 256, (64, 48, 3)).astype(np.float32) - 128.0)
    patches = Patcher().patch(img)                       # [h, w, c, 8, 8] view
    pq = PatchQuant()
    for h, w in ((0, 0), (3, 2), (7, 5)):
        blk3 = patches[h, w]                             # (3, 8, 8) view
        dct3 = np.zeros_like(blk3, dtype=np.float32)
        for c in range(3):
            dct3[c] = DCT.transform(blk3[c])             # non-contiguous (8, 8) float32
            assert_bits(DCT.transform(blk3[c]), O.dct_transform(np.ascontiguousarray(blk3[c])), "view")
        assert_bits(pq.quantize(dct3), O.quantize(dct3, 1.0), "E3-1 quantize")
    x = rng.normal(0, 50, (8, 8))
    ro = x.copy()
    ro.flags.writeable = False
    assert_bits(DCT.transform(ro), O.dct_transform(x), "read-only")
    sw = x.astype(">f8")                                  # not a kernel dtype: the general path
    assert_bits(DCT.transform(sw), O.dct_transform(x), "byte-swapped")
    one = rng.normal(0, 30, (1, 8, 8))
    assert_bits(pq.quantize(one), O.quantize(one, 1.0), "C = 1 stack")
    assert pq.quantize(one).shape == (1, 1, 3, 8, 8)
    many = rng.normal(0, 30, (2, 3, 1, 8, 8))
    assert_bits(pq.quantize(many), O.quantize(many, 1.0), "C = 1 batch")
    stk = rng.normal(0, 40, (3, 8, 8))
    pq2 = PatchQuant(0.5)
    before = pq2.quantize(stk)
    pq2.luminance[0, 0] = 3.0                             # edited in place
    want = np.round(stk / pq2.get_quantization_table()[None, None]).astype(np.int32)
    assert_bits(pq2.quantize(stk), want, "edited luminance")
    assert not np.array_equal(before, want)
    pq2.quantization_scale = np.float64(0.25)             # a NumPy scalar: float64 table
    want = np.round(stk / pq2.get_quantization_table()[None, None]).astype(np.int32)
    assert_bits(pq2.quantize(stk), want, "new scale")
    q = pq2.quantize(stk)
    assert_bits(pq2.dequantize(q), (q * pq2.get_quantization_table()[None, None]).astype(np.int32),
                "dequantize")
    # the table formed in the C step under NumPy's promotion (ivc_pyfast.c quant_lc) and the
    # tables it declines, each against NumPy's own table
    u8 = rng.integers(0, 256, (3, 8, 8)).astype(np.uint8)
    lum64 = rng.uniform(1, 90, (8, 8))
    for lum, chrom, sc, xin in [(None, None, 0.3, u8), (None, None, 3, stk.astype(np.float32)),
                                (lum64, None, 2, stk), (lum64, lum64, np.float64(0.7), u8),
                                (lum64.astype(np.int64), None, 0.5, stk),
                                (lum64.astype(np.int64) + 1, lum64.astype(np.int64) + 2, 1.5, u8),
                                (lum64.astype(np.int32) + 1, None, 1.0, stk),     # declined
                                (None, None, np.float32(0.8), stk.astype(np.float32))]:  # declined
        p = PatchQuant(sc, lum, chrom)
        t = p.get_quantization_table()
        want = np.round(xin / t[None, None]).astype(np.int32)
        assert_bits(p.quantize(xin), want, f"table {t.dtype} scale {sc!r} input {xin.dtype}")
        q = p.quantize(xin)
        assert_bits(p.dequantize(q), (q * t[None, None]).astype(np.int32), f"dequantize {t.dtype}")


def test_dct_golden(golden):
    d = golden("dct")
    assert_bits(DCT.transform(d["x_u8"]), d["dct_u8"], "dct u8")
    assert_bits(DCT.transform(d["x_f64"]), d["dct_f64"], "dct f64")
    assert_bits(DCT.inverse_transform(d["x_f64"]), d["idct_f64"], "idct f64")
    assert_bits(DCT.transform(d["x_f32"]), d["dct_f32"], "dct f32")
    assert_bits(DCT.inverse_transform(d["x_f32"]), d["idct_f32"], "idct f32")
    assert_bits(DCT.inverse_transform(d["x_i32"]), d["idct_i32"], "idct i32")
    assert_bits(DCT.transform(d["x_i16"]), d["dct_i16"], "dct i16")
    for norm in ("backward", "forward"):
        D2 = DiscreteCosineTransform(norm=norm)
        assert_bits(D2.transform(d["x_f64"][:64]), d[f"dct_f64_{norm}"], norm)
        assert_bits(D2.inverse_transform(d["x_f64"][:64]), d[f"idct_f64_{norm}"], norm)
    assert_bits(DCT.transform(Patcher().patch(d["x_img"])), d["dct_img"], "patched view")


@pytest.mark.parametrize("dtype", ALL_DTYPES + [np.float16, np.bool_])
def test_dct_dtypes_vs_oracle(dtype):
    rng = np.random.default_rng(11)
    if dtype == np.bool_:
        x = rng.integers(0, 2, (3, 5, 2, 8, 8)).astype(bool)
    else:
        x = rand_array(rng, dtype, (3, 5, 2, 8, 8))
    assert_bits(DCT.transform(x), O.dct_transform(x), f"dct {dtype}")
    assert_bits(DCT.inverse_transform(x), O.dct_inverse(x), f"idct {dtype}")


def test_dct_shapes_and_errors():
    rng = np.random.default_rng(3)
    b = rng.integers(0, 256, (8, 8)).astype(np.uint8)
    assert_bits(DCT.transform(b), O.dct_transform(b), "bare block")
    b3 = rng.normal(size=(3, 8, 8)).astype(np.float32)
    assert_bits(DCT.transform(b3), O.dct_transform(b3), "(3,8,8) float32")
    e = np.zeros((0, 4, 8, 8))
    assert DCT.transform(e).shape == (0, 4, 8, 8)
    nc = rng.normal(size=(4, 8, 8, 3)).transpose(0, 3, 1, 2)  # non-contiguous
    assert_bits(DCT.transform(nc), O.dct_transform(nc), "non-contiguous")
    c = rng.normal(size=(2, 8, 8)) + 1j * rng.normal(size=(2, 8, 8))
    assert np.array_equal(DCT.transform(c), O.dct_transform(c))
    with pytest.raises(ValueError):
        DiscreteCosineTransform(norm="bogus").transform(b)
    with pytest.raises(NotImplementedError):
        DCT.transform(np.zeros((16, 16)))
    with pytest.raises(ValueError):
        DCT.transform(np.zeros(8))


def test_dct_large_u8_roundtrip_property():
    """Full 4K luma frame: bit-exact vs the oracle, and IDCT(DCT(x)) ~= x."""
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (2160, 3840, 1), dtype=np.uint8)
    p = Patcher().patch(img)
    y = DCT.transform(p)
    assert_bits(y, O.dct_transform(p), "4K dct")
    assert np.allclose(DCT.inverse_transform(y), p, atol=1e-9)


# ------------------------------------------------------------------------ quantisation -
def test_quant_golden(golden):
    q = golden("quant")
    d1 = DCT.transform(Patcher().patch(q["img1"]))
    d3 = DCT.transform(Patcher().patch(q["img3"]))
    for i, s in enumerate(q["scales"]):
        Q = PatchQuant(quantization_scale=float(s))
        assert_bits(Q.get_quantization_table(), q[f"table_{i}"], "table")
        assert_bits(Q.quantize(d1), q[f"q1_{i}"], f"q1 scale {s}")
        assert_bits(Q.quantize(d3), q[f"q3_{i}"], f"q3 scale {s}")
        assert_bits(Q.dequantize(q[f"q1_{i}"]), q[f"dq1_{i}"], f"dq1 scale {s}")
        assert_bits(Q.dequantize(q[f"q3_{i}"]), q[f"dq3_{i}"], f"dq3 scale {s}")
        assert_bits(DCT.inverse_transform(q[f"dq3_{i}"]), q[f"idq3_{i}"], f"idq3 scale {s}")
    Q1 = PatchQuant(1.0)
    assert_bits(Q1.quantize(Patcher().patch(q["img3"])), q["raw_q3"], "raw pixels")
    assert_bits(Q1.dequantize(q["raw_q3"]), q["raw_dq3"], "raw dequant")
    assert_bits(Q1.quantize(q["f32_dct3"]), q["f32_q3"], "float32 dct")
    assert_bits(Q1.quantize(q["blk88"]), q["blk88_q"], "(8,8)")
    assert_bits(Q1.quantize(q["blk388"]), q["blk388_q"], "(3,8,8)")
    assert_bits(Q1.quantize(q["ties_in"]), q["ties_q"], "ties")


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.uint8, np.int16, np.int32,
                                   np.int64, np.uint64, np.float16, np.bool_])
@pytest.mark.parametrize("scale", [1.0, 0.07, 2.5])
def test_quant_dequant_dtypes_vs_oracle(dtype, scale):
    rng = np.random.default_rng(int(scale * 100))
    shape = (4, 6, 1, 8, 8) if dtype in (np.uint8, np.int16) else (4, 6, 3, 8, 8)
    x = rng.integers(0, 2, shape).astype(bool) if dtype == np.bool_ else rand_array(rng, dtype, shape)
    assert_bits(PatchQuant(scale).quantize(x), O.quantize(x, scale), f"quantize {dtype}")
    assert_bits(PatchQuant(scale).dequantize(x), O.dequantize(x, scale), f"dequantize {dtype}")


def test_quant_scale_dtypes():
    """A NumPy float64 scale makes a float64 table (NumPy 2 promotion) — follow it."""
    rng = np.random.default_rng(9)
    x = rng.normal(0, 300, (2, 2, 3, 8, 8)).astype(np.float32)
    for s in (np.float64(0.3), np.float32(0.3), 3):
        Q = PatchQuant(s)
        ref = np.round(x / Q.get_quantization_table()[None, None]).astype(np.int32)
        assert_bits(Q.quantize(x), ref, f"scale {type(s)}")
        refd = (x * Q.get_quantization_table()[None, None]).astype(np.int32)
        assert_bits(Q.dequantize(x), refd, f"dequant scale {type(s)}")


def test_quant_broadcast_and_errors():
    Q = PatchQuant(0.5)
    rng = np.random.default_rng(2)
    for shape in [(8, 8), (3, 8, 8), (1, 8, 8), (2, 3, 1, 8, 8), (5, 1, 1, 3, 8, 8), (1, 8), (),
                  (4, 4, 3, 1, 8)]:
        x = rng.normal(0, 100, shape)
        assert_bits(Q.quantize(x), O.quantize(x, 0.5), f"broadcast {shape}")
    with pytest.raises(ValueError):
        Q.quantize(np.zeros((4, 4, 2, 8, 8)))
    x = np.array([np.nan, np.inf, -np.inf, 1e12, -1e12, 0.5 * 16, 1.5 * 16, 2.5 * 16] * 8)
    x = x.reshape(1, 1, 1, 8, 8)
    assert_bits(Q.quantize(x), O.quantize(x, 0.5), "non-finite / out of range")
    assert_bits(Q.dequantize(np.full((1, 1, 3, 8, 8), 2**30, np.int32)),
                O.dequantize(np.full((1, 1, 3, 8, 8), 2**30, np.int32), 0.5), "dequant overflow")


# ------------------------------------------------------------------------ zig-zag ------
def test_zigzag_golden(golden):
    z = golden("zigzag")
    Z = ZigZag()
    assert np.array_equal(Z.zigzag_order, z["order"])
    assert_bits(Z.flatten(z["x5"]), z["flat"], "flatten")
    assert_bits(Z.unflatten(z["flat"]), z["unflat"], "unflatten")
    assert_bits(Z.flatten(z["x5_f64"]), z["flat_f64"], "flatten f64")
    assert_bits(Z.flatten(z["x5_i16"]), z["flat_i16"], "flatten i16")
    assert_bits(zigzag_scan(z["blk"]), z["scan"], "zigzag_scan")


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.int32, np.float64, np.complex64])
def test_zigzag_dtypes_and_shapes(dtype):
    rng = np.random.default_rng(4)
    x = rng.integers(-100, 100, (3, 4, 2, 8, 8)).astype(dtype)
    Z = ZigZag()
    f = Z.flatten(x)
    assert_bits(f, O.zigzag_flatten(x), f"flatten {dtype}")
    assert_bits(Z.unflatten(f), x, f"roundtrip {dtype}")
    wide = rng.integers(-100, 100, (2, 2, 1, 70)).astype(dtype)   # rows wider than 64
    assert_bits(Z.unflatten(wide), O.zigzag_unflatten(wide), "unflatten wide rows")
    assert_bits(Z.flatten(x.reshape(3, 4, 2, 4, 16)), O.zigzag_flatten(x.reshape(3, 4, 2, 4, 16)), "4x16")
    assert Z.flatten(np.zeros((0, 2, 3, 8, 8), dtype)).shape == (0, 2, 3, 64)
    with pytest.raises(AssertionError):
        zigzag_scan(np.zeros((4, 4)))


# ------------------------------------------------------------------------ motion -------
ME_CASES = ["shift_f64_sr4", "shift_f64_sr16", "flat_sr4", "nonint_f64_sr4", "f32_sr4",
            "u8mod_sr4", "u8mod_sr7", "i16_sr4", "i32_sr3", "periodic_f64_sr8",
            "periodic_f32_sr8", "periodic2_f64_sr5"]


@pytest.mark.parametrize("case", ME_CASES)
def test_me_golden(golden, case):
    m = golden("motion")
    ref, cur, sr = m[f"{case}_ref"], m[f"{case}_cur"], int(m[f"{case}_sr"])
    mv = MotionCompensator(sr).compute_motion_vector(ref, cur)
    assert_bits(mv, m[f"{case}_mv"], case)


@pytest.mark.parametrize("dtype", ALL_DTYPES)
def test_me_dtypes_vs_c_oracle(dtype):
    rng = np.random.default_rng(21)
    base = rand_array(rng, dtype, (80, 96))
    cur = np.roll(base, (2, -3), axis=(0, 1))
    cur[::7] = rand_array(rng, dtype, cur[::7].shape)
    for sr in (0, 3, 9):
        mv = MotionCompensator(sr).compute_motion_vector(base, cur)
        assert_bits(mv, c_motion_vectors(base, cur, sr), f"{dtype} sr={sr}")


def test_me_large_search_vs_c_oracle():
    rng = np.random.default_rng(8)
    a = rng.normal(128, 50, (144, 176))                    # QCIF, non-integer float64
    b = np.roll(a, (5, -7), axis=(0, 1)) + rng.normal(0, 0.5, a.shape)
    for sr in (16, 23):
        assert_bits(MotionCompensator(sr).compute_motion_vector(a, b), c_motion_vectors(a, b, sr),
                    f"sr={sr}")


def test_me_exact_u8_mode_and_mixed_dtypes():
    import ivclab_amd._native as N
    rng = np.random.default_rng(12)
    a = rng.integers(0, 256, (64, 80), dtype=np.uint8)
    b = np.roll(a, (-4, 6), axis=(0, 1))
    want = O.motion_vectors(a.astype(np.float64), b.astype(np.float64), 8)
    mv = np.empty((8, 10, 1), np.int64)
    N.check(N.lib().ivc_motion_estimate(N.ptr(a), N.ptr(b), 1, 1, 64, 80, 8, N.ME_EXACT_U8, N.ptr(mv)))
    assert_bits(mv, want, "exact-u8 mode")
    assert_bits(MotionCompensator(8).compute_motion_vector(a.astype(np.float64), b), want, "f64 vs u8")


def test_me_errors():
    M = MotionCompensator(4)
    with pytest.raises(ValueError):
        M.compute_motion_vector(np.zeros((12, 16)), np.zeros((12, 16)))
    with pytest.raises(TypeError):
        M.compute_motion_vector(np.zeros((8, 8), bool), np.zeros((8, 8), bool))


def test_mc_golden(golden):
    m = golden("motion")
    M = MotionCompensator(4)
    assert_bits(M.reconstruct_with_motion_vector(m["mc_ref1"], m["mc_mv"]), m["mc_out1"], "mc f64")
    assert_bits(M.reconstruct_with_motion_vector(m["mc_ref3"], m["mc_mv"]), m["mc_out3"], "mc u8x3")


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.float32, np.float64])
def test_mc_random_vs_c_oracle(dtype):
    rng = np.random.default_rng(30)
    sr = 5
    ref = rand_array(rng, dtype, (48, 64, 2))
    mv = rng.integers(-20, (2 * sr + 1) ** 2 + 20, (6, 8, 1))   # includes out-of-range indices
    got = MotionCompensator(sr).reconstruct_with_motion_vector(ref, mv)
    assert_bits(got, c_motion_compensate(ref, mv[..., 0], sr), f"mc {dtype}")
    assert_bits(got, O.motion_compensate(ref, mv, sr), f"mc {dtype} (python)")


# ------------------------------------------------------------------------ fused paths --
def _native():
    import ivclab_amd._native as N
    return N, N.lib()


@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("zz", [0, 1])
def test_intra_encode_golden(golden, C, zz):
    N, L = _native()
    p = golden("intra")
    img = np.ascontiguousarray(p[f"img{C}"])
    H, W, _ = img.shape
    t = N.table_arg(PatchQuant(0.5).get_quantization_table())
    out = np.empty((H // 8, W // 8, 3, 64), np.int32)
    N.check(L.ivc_intra_encode(N.ptr(img), 1, 1, H, W, C, N.ptr(t), N.F64, zz, N.ptr(out)))
    want = p[f"zz{C}"] if zz else p[f"q{C}"].reshape(H // 8, W // 8, 3, 64)
    assert_bits(out, want, f"intra C={C} zz={zz}")
    rec = np.empty((H // 8 * W // 8, 3, 64), np.float64)
    N.check(L.ivc_intra_decode(N.ptr(p[f"zz{C}"]), (H // 8) * (W // 8), N.ptr(t), N.F64, 1, N.ptr(rec)))
    assert_bits(rec.reshape(H // 8, W // 8, 3, 8, 8), p[f"rec{C}"], "intra decode")


@pytest.mark.parametrize("scale", [1.0, 0.5, 0.15, 2.0, 0.07, 0.013])
@pytest.mark.parametrize("dtype", [np.uint8, np.float32, np.float64])
def test_intra_encode_vs_oracle(scale, dtype):
    N, L = _native()
    rng = np.random.default_rng(int(scale * 1000) + 1)
    F, H, W, C = 2, 72, 264, (1 if dtype == np.uint8 else 3)  # w = 33 blocks: ragged tile
    if dtype == np.uint8:
        img = rng.integers(0, 256, (F, H, W, C), dtype=np.uint8)
        img[:, :16] = img[:, :1, :1]                          # flat region: DC ties
    else:
        img = rng.normal(128, 60, (F, H, W, C)).astype(dtype)
    table = PatchQuant(scale).get_quantization_table()
    t = N.table_arg(table)
    calc = N.F32 if (dtype == np.float32 and table.dtype == np.float32) else N.F64
    out = np.empty((F, H // 8, W // 8, 3, 64), np.int32)
    N.check(L.ivc_intra_encode(N.ptr(img), N.DTYPE_CODE[np.dtype(dtype)], F, H, W, C, N.ptr(t),
                               calc, 1, N.ptr(out)))
    for f in range(F):
        assert_bits(out[f], O.intra_encode(img[f], scale, zigzag=True), f"frame {f}")


@pytest.mark.parametrize("dtype", [np.uint8, np.float64])
@pytest.mark.parametrize("zz", [0, 1])
def test_intra_encode_distinct_chroma_planes(dtype, zz):
    """A C-ABI table whose planes 1 and 2 differ (PatchQuant never builds one): the C = 1
    kernels then stage and quantise all three planes instead of storing plane 1 twice."""
    N, L = _native()
    rng = np.random.default_rng(12)
    F, H, W = 2, 48, 136
    img = (rng.integers(0, 256, (F, H, W, 1), dtype=np.uint8) if dtype == np.uint8
           else rng.normal(128, 60, (F, H, W, 1)))
    table = PatchQuant(0.5).get_quantization_table().astype(np.float64)
    table[2] *= 1.37
    out = np.empty((F, H // 8, W // 8, 3, 64), np.int32)
    N.check(L.ivc_intra_encode(N.ptr(img), N.DTYPE_CODE[np.dtype(dtype)], F, H, W, 1,
                               N.ptr(N.table_arg(table)), N.F64, zz, N.ptr(out)))
    for f in range(F):
        want = np.round(O.dct_transform(O.patch(img[f])) / table[None, None]).astype(np.int32)
        want = O.zigzag_flatten(want) if zz else want.reshape(H // 8, W // 8, 3, 64)
        assert_bits(out[f], want, f"frame {f}")


def test_cfg1_512_gray_through_the_classes():
    """BASELINE configs[0] (default_rng(0), 512x512x1 u8): Patcher.patch ->
    DCT.transform -> PatchQuant.quantize through the drop-in classes, and the fused kernel,
    bit-exact against the oracle; then dequantize -> inverse_transform -> unpatch."""
    N, L = _native()
    img = np.random.default_rng(0).integers(0, 256, (512, 512, 1), dtype=np.uint8)
    P, D, Q = Patcher(), DiscreteCosineTransform(), PatchQuant(1.0)
    q = Q.quantize(D.transform(P.patch(img)))
    want = O.quantize(O.dct_transform(O.patch(img)), 1.0)
    assert q.shape == (64, 64, 3, 8, 8)
    assert_bits(q, want, "cfg1 classes")
    t = N.table_arg(Q.get_quantization_table())
    fused = np.empty((1, 64, 64, 3, 64), np.int32)
    N.check(L.ivc_intra_encode(N.ptr(np.ascontiguousarray(img[None])), 1, 1, 512, 512, 1, N.ptr(t),
                               N.F64, 0, N.ptr(fused)))
    assert_bits(fused[0], want.reshape(64, 64, 3, 64), "cfg1 fused")
    rec = P.unpatch(D.inverse_transform(Q.dequantize(q)))
    assert_bits(rec, O.unpatch(O.dct_inverse(O.dequantize(want, 1.0))), "cfg1 inverse")


def test_cfg2_1080p_rgb_per_channel_with_zigzag():
    """BASELINE configs[1] (default_rng(1), 1920x1080 RGB u8): per-channel DCT +
    quantise + zig-zag through the classes and the fused kernel (C = 3), bit-exact."""
    N, L = _native()
    img = np.random.default_rng(1).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
    P, D, Q, Z = Patcher(), DiscreteCosineTransform(), PatchQuant(1.0), ZigZag()
    zz = Z.flatten(Q.quantize(D.transform(P.patch(img))))
    want = O.zigzag_flatten(O.quantize(O.dct_transform(O.patch(img)), 1.0))
    assert zz.shape == (135, 240, 3, 64)
    assert_bits(zz, want, "cfg2 classes")
    t = N.table_arg(Q.get_quantization_table())
    fused = np.empty((1, 135, 240, 3, 64), np.int32)
    N.check(L.ivc_intra_encode(N.ptr(np.ascontiguousarray(img[None])), 1, 1, 1080, 1920, 3, N.ptr(t),
                               N.F64, 1, N.ptr(fused)))
    assert_bits(fused[0], want, "cfg2 fused")


def test_intra_encode_4k_full_frame():
    """One full cfg3 frame (3840x2160 luma) bit-exact against the oracle."""
    N, L = _native()
    rng = np.random.default_rng(2160)
    img = rng.integers(0, 256, (1, 2160, 3840, 1), dtype=np.uint8)
    img[0, 1000:1200] = 77
    t = N.table_arg(PatchQuant(1.0).get_quantization_table())
    out = np.empty((1, 270, 480, 3, 64), np.int32)
    N.check(L.ivc_intra_encode(N.ptr(img), 1, 1, 2160, 3840, 1, N.ptr(t), N.F64, 0, N.ptr(out)))
    want = O.intra_encode(img[0], 1.0).reshape(270, 480, 3, 64)
    assert_bits(out[0], want, "4K intra")


@pytest.mark.parametrize("zz", [False, True])
@pytest.mark.parametrize("scale", [1.0, 0.013])
def test_intra_encode_luma_only_vs_oracle(zz, scale):
    """ivc_intra_encode_luma_dev: plane 0 (the luminance table) of the reference's 3-plane
    quantisation of a grayscale batch, [F, h, w, 64] int32; ragged groups (w = 33 blocks) and
    a fine scale (magnitude-checked quotients)."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(int(zz) + 7)
    F, H, W = 3, 72, 264
    img = rng.integers(0, 256, (F, H, W), dtype=np.uint8)
    img[:, :16] = 77
    table = PatchQuant(scale).get_quantization_table()
    out = torch.full((F, H // 8, W // 8, 64), -5, dtype=torch.int32, device="cuda")
    D.intra_encode_luma(torch.from_numpy(img).cuda(), table, out, zigzag=zz)
    torch.cuda.synchronize()
    for f in range(F):
        want = O.intra_encode(img[f][..., None], scale, zigzag=zz)[:, :, 0].reshape(H // 8, W // 8, 64)
        assert_bits(out[f].cpu().numpy(), want, f"luma-only frame {f}")


def test_store_pacing_changes_timing_only():
    """Paced launches (8 4K frames: every wave stores >= 8 slots, so the clock schedule is
    live) give the same bytes as unpaced ones at any rate — far too fast (every slot late),
    adaptive default, far too slow (every wave waits) — and the pace API reports the rate and
    the late fraction it adapts from.  Frame 0 is checked against the oracle."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    N, L = _native()
    rng = np.random.default_rng(88)
    F, H, W = 8, 2160, 3840
    img = rng.integers(0, 256, (F, H, W, 1), dtype=np.uint8)
    img[:, 500:700] = 31                                        # flat rows: DC ties
    x = torch.from_numpy(img).cuda()
    table = PatchQuant(1.0).get_quantization_table()
    outs = {}
    start = L.ivc_store_pace()
    try:
        for rate in (0.0, 1e6, 5800.0, 600.0):
            N.check(L.ivc_set_store_pace(rate))
            assert L.ivc_store_pace() == rate
            o = torch.full((F, H // 8, W // 8, 3, 64), -7, dtype=torch.int32, device="cuda")
            for _ in range(3):                                  # adaptive steps in between
                D.intra_encode(x, table, o)
            torch.cuda.synchronize()
            outs[rate] = o.cpu().numpy()
            late = L.ivc_store_pace_late()
            assert late == -1.0 or 0.0 <= late <= 1.0
        assert L.ivc_set_store_pace(-1.0) == N.E_ARG
    finally:
        N.check(L.ivc_set_store_pace(start))
    for rate, o in outs.items():
        assert_bits(o, outs[0.0], f"paced at {rate} GB/s")
    want = O.intra_encode(img[0], 1.0).reshape(H // 8, W // 8, 3, 64)
    assert_bits(outs[5800.0][0], want, "paced 4K frame 0")


def test_store_pace_trace_settle_and_threads():
    """The pacing controller's per-launch trace and settle (include/ivc.h): a rate far above
    any device's (every slot late) is stepped back from THAT launch's rate — a burst of such
    launches folded together does not compound — and settle never raises the rate.  Two host
    threads launching on two streams reserve distinct measurement slots: every launch is
    measured exactly once.  Outputs stay those of the oracle throughout."""
    torch = pytest.importorskip("torch")
    import threading
    import ivclab_amd.device as D
    N, L = _native()
    rng = np.random.default_rng(89)
    F, H, W = 8, 2160, 3840
    img = rng.integers(0, 256, (F, H, W, 1), dtype=np.uint8)
    x = torch.from_numpy(img).cuda()
    table = PatchQuant(1.0).get_quantization_table()
    start = L.ivc_store_pace()
    try:
        o = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device="cuda")
        D.intra_encode(x, table, o)                    # the process's first measured launch
        torch.cuda.synchronize()
        N.check(L.ivc_set_store_pace(50000.0))
        N.check(L.ivc_store_pace_reset_stats())
        for _ in range(4):                              # one burst, no synchronisation
            D.intra_encode(x, table, o)
        torch.cuda.synchronize()
        tr = N.pace_trace()
        assert len(tr) == 4
        assert all(r[0] == 50000.0 for r in tr), tr     # all ran at the rate set before them
        assert all(r[1] > 0.5 for r in tr), tr          # far too fast: most slots late
        # no compounding: every fold steps back from 50000 once (to <= 0.98 x 50000 or 1.1x
        # what the launch moved), never 0.98^k
        after = L.ivc_store_pace()
        assert 100.0 <= after <= 0.98 * 50000.0
        assert after >= min(1.1 * r[2] for r in tr) * 0.999, (after, tr)
        st = N.pace_stats()
        assert st["launches_measured"] == 4 and st["launches_over_late_threshold"] == 4
        before = L.ivc_store_pace()
        N.check(L.ivc_store_pace_settle(0.02))
        assert L.ivc_store_pace() <= before
        assert L.ivc_store_pace_settle(0.7) == N.E_ARG
        # two threads, two streams
        N.check(L.ivc_set_store_pace(5000.0))
        N.check(L.ivc_store_pace_reset_stats())
        outs = [torch.empty_like(o) for _ in range(2)]
        errs = []

        def worker(i):
            try:
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    for _ in range(3):
                        D.intra_encode(x, table, outs[i], stream=s)
                s.synchronize()
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        assert not errs, errs
        st = N.pace_stats()
        assert st["launches_measured"] == 6, st
        assert all(r[2] > 0 for r in N.pace_trace()), N.pace_trace()
    finally:
        N.check(L.ivc_set_store_pace(start))
    want = O.intra_encode(img[0], 1.0).reshape(H // 8, W // 8, 3, 64)
    for oo in [o] + outs:
        assert_bits(oo[0].cpu().numpy(), want, "paced 4K frame 0")


def test_pinned_host_pool_and_staging():
    """ivc_host_alloc blocks back the drop-in classes' large results (ivclab_amd._native.empty):
    a freed block is reused for the next array of that size, a foreign pointer is refused,
    and host-buffer calls give identical results from pinned and from pageable buffers, for
    transfers that take the direct DMA, the pinned ring (several 8 MiB chunks, H2D and D2H)
    and the small pageable path."""
    import gc
    N, L = _native()
    a = N.empty((1024, 1024), np.float64)
    p = a.ctypes.data
    assert not a.flags.owndata and a.flags.writeable
    del a
    gc.collect()
    b = N.empty((1024, 1024), np.float64)
    assert b.ctypes.data == p
    assert L.ivc_host_free(None) == 0
    assert L.ivc_host_free(p + 64) == N.E_ARG
    rng = np.random.default_rng(3)
    for nblk in (100, 40_000, 300_000):                  # 0.05, 20 and 150 MB of float64 out
        src = rng.integers(0, 256, (nblk, 64), dtype=np.uint8)
        want = O.dct_transform(src.reshape(nblk, 8, 8).astype(np.float64))
        for out in (np.empty((nblk, 8, 8)), N.empty((nblk, 8, 8), np.float64)):
            N.check(L.ivc_dct8x8(N.ptr(src), 1, nblk, N.ptr(out), N.F64, 0, 1))
            assert_bits(out, want, f"dct {nblk} blocks")
        # float64 input through the ring (H2D chunks), pinned and pageable
        srcf = src.astype(np.float64)
        for inp in (srcf, N.empty(srcf.shape, np.float64)):
            inp[...] = srcf
            out = N.empty((nblk, 8, 8), np.float64)
            N.check(L.ivc_dct8x8(N.ptr(inp), N.F64, nblk, N.ptr(out), N.F64, 0, 1))
            assert_bits(out, want, f"dct f64 in {nblk} blocks")


def test_histogram_vs_oracle():
    N, L = _native()
    rng = np.random.default_rng(1)
    sym = rng.integers(-3000, 3000, 1 << 20).astype(np.int32)
    sym[::3] = 0
    for lo, nb in ((-2048, 4096), (-40000, 70000)):
        h = np.zeros(nb, np.int64)
        N.check(L.ivc_histogram_i32(N.ptr(sym), sym.size, lo, nb, N.ptr(h)))
        assert np.array_equal(h, O.histogram(sym, lo, nb))


def test_histogram_occupancy_changes_timing_only():
    """ivc_set_histogram_occupancy (workgroups per CU) leaves the counts unchanged, on the
    caller's stream next to another stream's work; 0 restores the default, > 16 is refused."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    N, L = _native()
    rng = np.random.default_rng(5)
    sym = rng.integers(-300, 300, (1 << 22) + 3).astype(np.int32)
    sym[::2] = 0
    want = O.histogram(sym, -2048, 4096)
    s = torch.from_numpy(sym).cuda()
    side = torch.cuda.Stream()
    start = L.ivc_histogram_occupancy()
    try:
        for k in (1, 2, 16, 0):
            N.check(L.ivc_set_histogram_occupancy(k))
            assert L.ivc_histogram_occupancy() == (k or 4)
            h = torch.zeros(4096, dtype=torch.int64, device="cuda")
            side.wait_stream(torch.cuda.current_stream())
            D.histogram(s, -2048, h, stream=side)
            torch.cuda.current_stream().wait_stream(side)
            assert np.array_equal(h.cpu().numpy(), want), k
        assert L.ivc_set_histogram_occupancy(17) == N.E_ARG
        assert L.ivc_set_histogram_occupancy(-1) == N.E_ARG
    finally:
        N.check(L.ivc_set_histogram_occupancy(start))


def test_histogram_i64_vs_oracle():
    """int64 symbols (motion-vector indices): host entry point, values beyond both ends."""
    N, L = _native()
    rng = np.random.default_rng(3)
    sym = rng.integers(-50, 1200, (1 << 18) + 5).astype(np.int64)
    sym[::7] = 0
    sym[:4] = [-(1 << 62), 1 << 62, np.iinfo(np.int64).min + 1, np.iinfo(np.int64).max]
    for lo, nb in ((0, 1089), (-64, 2048), (-40000, 70000)):
        h = np.zeros(nb, np.int64)
        N.check(L.ivc_histogram_i64(N.ptr(sym), sym.size, lo, nb, N.ptr(h)))
        want = O.histogram(np.clip(sym, lo - 1, lo + nb + 1), lo, nb)
        assert np.array_equal(h, want), (lo, nb)


@pytest.mark.parametrize("dt", ["int32", "int64"])
def test_histogram_device_offsets_and_ragged(dt):
    """Device histogram on views that start off 16 B and lengths that are not multiples of
    the 16-byte vector (the kernel reads 16 B per lane after an unaligned head)."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(2)
    base = rng.integers(-300, 300, (1 << 16) + 9).astype(dt)
    base[::5] = 0
    t = torch.from_numpy(base).cuda()
    for off in (0, 1, 2, 3):
        for n in (0, 1, 3, 4, 5, 7, 1023, 4096 + 3, base.size - off):
            h = torch.zeros(512, dtype=torch.int64, device="cuda")
            D.histogram(t[off:off + n], -256, h)
            assert np.array_equal(h.cpu().numpy(), O.histogram(base[off:off + n], -256, 512)), (off, n)
    # the register-counted values -3..4 landing in clamped end bins, bins starting inside them,
    # a one-bin histogram, and more than 16384 bins (global atomics instead of LDS)
    hot = rng.integers(-6, 8, 1 << 18).astype(dt)
    th = torch.from_numpy(hot).cuda()
    for lo, nb in ((2, 3), (-1, 2), (0, 1), (-3, 8), (-100, 20000), (5, 4)):
        h = torch.zeros(nb, dtype=torch.int64, device="cuda")
        D.histogram(th, lo, h)
        assert np.array_equal(h.cpu().numpy(), O.histogram(hot, lo, nb)), (lo, nb)


# ------------------------------------------------------------------------ device API ---
def test_device_api_intra_and_inter():
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(77)
    F, H, W, sr = 4, 64, 96, 7
    base = rng.integers(0, 256, (H + 32, W + 32), dtype=np.uint8)
    frames = np.stack([base[(f % 3):(f % 3) + H, (2 * f % 5):(2 * f % 5) + W] for f in range(F)])
    frames[2, 10:20, 30:50] = rng.integers(0, 256, (10, 20))
    dev = torch.device("cuda:0")
    tf = torch.from_numpy(frames).to(dev)
    table = PatchQuant(1.0).get_quantization_table()
    mv = torch.empty((F - 1, H // 8, W // 8), dtype=torch.int64, device=dev)
    out = torch.empty((F - 1, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    D.inter_encode(tf, sr, table, mv, out)
    qi = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    hist = torch.zeros(8192, dtype=torch.int64, device=dev)
    D.intra_encode(tf[..., None].contiguous(), table, qi, zigzag=True, hist=hist, hist_lo=-4096)
    torch.cuda.synchronize()
    mv, out, qi, hist = mv.cpu().numpy(), out.cpu().numpy(), qi.cpu().numpy(), hist.cpu().numpy()
    for f in range(1, F):
        wmv, wq = O.inter_encode(frames[f - 1], frames[f], sr, 1.0)
        assert_bits(mv[f - 1], wmv[..., 0].astype(np.int64), f"inter mv {f}")
        assert_bits(out[f - 1], wq.reshape(H // 8, W // 8, 3, 64), f"inter q {f}")
    for f in range(F):
        assert_bits(qi[f], O.intra_encode(frames[f][..., None], 1.0, zigzag=True), f"intra {f}")
    assert np.array_equal(hist, O.histogram(qi, -4096, 8192))


@pytest.mark.parametrize("sr", [4, 8, 16, 5])
@pytest.mark.parametrize("shape", [(16, 16), (72, 264), (136, 120), (8, 224)])
def test_me_exact_u8_fast_paths(sr, shape):
    """Exact-u8 mode (fast dot4 kernel for sr in {4, 8, 16}, generic otherwise) against the
    C oracle on the float64 frames: random, shifted, flat (all-tie) and edge-heavy sizes."""
    import ivclab_amd._native as N
    rng = np.random.default_rng(sr * 1000 + shape[1])
    H, W = shape
    base = rng.integers(0, 256, (H + 40, W + 40), dtype=np.uint8)
    cases = [(base[:H, :W], base[3:H + 3, 5:W + 5]),
             (np.full((H, W), 77, np.uint8), np.full((H, W), 77, np.uint8)),
             (base[:H, :W], np.zeros((H, W), np.uint8))]
    for ref, cur in cases:
        ref, cur = np.ascontiguousarray(ref), np.ascontiguousarray(cur)
        mv = np.empty((H // 8, W // 8, 1), np.int64)
        N.check(N.lib().ivc_motion_estimate(N.ptr(ref), N.ptr(cur), 1, 1, H, W, sr, N.ME_EXACT_U8, N.ptr(mv)))
        want = c_motion_vectors(ref.astype(np.float64), cur.astype(np.float64), sr)
        assert_bits(mv, want.astype(np.int64), f"exact u8 sr={sr} {shape}")


@pytest.mark.parametrize("sr", [4, 8, 16])
@pytest.mark.parametrize("shape", [(88, 200), (40, 136), (24, 48)])
def test_me_exact_u8_extremes_multi_frame(sr, shape):
    """Several frame pairs in one call (the tiled sr=16 kernel's tiles cross frames), with
    extreme contrast: binary 0/255 content (SSDs up to 64 * 255^2, the top of the key range),
    all-255 against all-0 (every candidate ties at the maximum), and mixed — against the C
    oracle, frame by frame."""
    import ivclab_amd._native as N
    rng = np.random.default_rng(sr * 7 + shape[1])
    H, W = shape
    binary = (rng.integers(0, 2, (H + 40, W + 40)) * 255).astype(np.uint8)
    refs = [binary[:H, :W], np.full((H, W), 255, np.uint8), rng.integers(0, 256, (H, W), dtype=np.uint8),
            binary[5:H + 5, 2:W + 2]]
    curs = [binary[2:H + 2, 6:W + 6], np.zeros((H, W), np.uint8), np.full((H, W), 255, np.uint8),
            np.flipud(binary[:H, :W])]
    ref = np.ascontiguousarray(np.stack(refs))
    cur = np.ascontiguousarray(np.stack(curs))
    F = ref.shape[0]
    mv = np.empty((F, H // 8, W // 8, 1), np.int64)
    N.check(N.lib().ivc_motion_estimate(N.ptr(ref), N.ptr(cur), 1, F, H, W, sr, N.ME_EXACT_U8, N.ptr(mv)))
    for f in range(F):
        want = c_motion_vectors(ref[f].astype(np.float64), cur[f].astype(np.float64), sr)
        assert_bits(mv[f], want.astype(np.int64), f"extremes sr={sr} {shape} frame {f}")


def test_me_exact_u8_full_hd_vs_c_oracle():
    """A full 1080p pair at sr=16 (the bench configuration), checked on sampled block rows
    (top, middle, bottom) against the C oracle."""
    import ivclab_amd._native as N
    rng = np.random.default_rng(1080)
    lo = rng.integers(0, 256, (290, 500)).astype(np.float64)
    big = np.kron(lo, np.ones((4, 4)))[:1120, :1960] + rng.integers(-8, 9, (1120, 1960))
    big = np.clip(big, 0, 255).astype(np.uint8)
    ref, cur = np.ascontiguousarray(big[:1080, :1920]), np.ascontiguousarray(big[3:1083, 7:1927])
    mv = np.empty((135, 240, 1), np.int64)
    N.check(N.lib().ivc_motion_estimate(N.ptr(ref), N.ptr(cur), 1, 1, 1080, 1920, 16, N.ME_EXACT_U8, N.ptr(mv)))
    for rows in ((0, 3), (66, 69), (132, 135)):
        want = c_motion_vectors(ref, cur, 16, exact_u8=True, rows=rows)
        assert_bits(mv[rows[0]:rows[1]], want.astype(np.int64), f"1080p rows {rows}")


# ------------------------------------------------------------------- zero-run coding ---
ZR_ENC = ["zz1", "zz3", "sparse", "eob1000", "bs16"]
ZR_ERR = ["truncated", "trailing_zero", "truncated_mid", "ends_after_zero", "ends_after_zero2",
          "overflow", "overflow_run", "too_few", "extra_ignored", "negative_run",
          "early_eob_value", "empty", "zero_blocks"]


@pytest.mark.parametrize("case", ZR_ENC)
def test_zerorun_encode_golden(golden, case):
    from ivclab_amd.entropy import ZeroRunCoder
    z = golden("zerorun")
    Z = ZeroRunCoder(int(z[f"{case}_eob"]), int(z[f"{case}_bs"]))
    assert_bits(Z.encode(z[f"{case}_x"]), z[f"{case}_sym"], case)


def test_zerorun_decode_golden(golden):
    from ivclab_amd.entropy import ZeroRunCoder
    z = golden("zerorun")
    Z = ZeroRunCoder()
    assert_bits(Z.decode(z["sparse_sym"], z["sparse_x"].shape[:3]), z["dec_sparse"], "sparse")
    assert_bits(Z.decode(z["zz3_sym"], z["zz3_x"].shape[:3]), z["dec_zz3"], "zz3")


@pytest.mark.parametrize("case", ZR_ERR)
def test_zerorun_decode_errors_golden(golden, case):
    from ivclab_amd.entropy import ZeroRunCoder
    z = golden("zerorun")
    sym, shape = z[f"err_{case}_sym"], tuple(int(v) for v in z[f"err_{case}_shape"])
    exc = str(z[f"err_{case}_exc"])
    if exc:
        with pytest.raises(Exception) as ei:
            ZeroRunCoder().decode(sym, shape)
        assert f"{type(ei.value).__name__}: {ei.value}" == exc
    else:
        assert_bits(ZeroRunCoder().decode(sym, shape), z[f"err_{case}_out"], case)


def test_zerorun_decode_fast_path_boundaries():
    """The fast decoder (ivc_entropy.hip zf_*: local slot typing, 4096-symbol tiles, a
    128-symbol halo) against the oracle on streams built to stress it: the longest blocks
    (97 symbols: alternating value / zero-run, crossing tile boundaries), all-EOB stretches
    longer than the halo, coefficient values equal to the EOB symbol and to the run lengths,
    and streams it must hand to the general decoder (a zero run-length after a zero value,
    a negative run, an overflowing block, trailing garbage after the expected blocks, too few
    blocks, a stream ending after a zero) — results and errors identical either way."""
    from ivclab_amd.entropy import ZeroRunCoder
    rng = np.random.default_rng(97)
    Z = ZeroRunCoder()
    nb = 3000
    x = np.zeros((nb, 64), np.int32)
    kinds = rng.integers(0, 5, nb)
    for i, k in enumerate(kinds):
        if k == 0:                                         # longest: v 0 run, repeated
            x[i, 0::2] = rng.integers(1, 9, 32) * rng.choice([-1, 1], 32)
        elif k == 1:
            pass                                           # all-zero: EOB only
        elif k == 2:
            x[i] = rng.integers(-3, 4, 64)
        elif k == 3:
            x[i, rng.integers(0, 64, 3)] = 4000            # the EOB value as a coefficient
        else:
            x[i, :8] = rng.integers(1, 64, 8)              # values equal to run lengths
    x[1000:1400] = 0                                       # 400 EOBs in a row (> halo)
    sym = O.zerorun_encode_fast(x)
    shape = (nb // 30, 30, 1)
    assert sym.size > 3 * 4096
    # (the EOB symbol as a coefficient decodes as an EOB in the reference: the stream is then
    # parsed as the reference parses it, whatever that yields)
    bad = {
        "clean": sym,
        "clean_no_eob_values": O.zerorun_encode_fast(np.where(x == 4000, 4001, x)),
        "zero_run_zero": np.concatenate([sym[:50], [0, 0, 5], sym[50:]]),
        "negative_run": np.concatenate([sym[:50], [0, -2], sym[50:]]),
        "overflow": np.concatenate([[0, 63, 7, 7], sym]),
        "trailing_garbage": np.concatenate([sym, [0, 0, 0, -5, 4000]]),
        "too_few": sym[: np.flatnonzero(sym == 4000)[nb // 2]],
        "ends_after_zero": np.concatenate([sym[: np.flatnonzero(sym == 4000)[10] + 1], [5, 0]]),
    }
    k10 = int(np.flatnonzero(sym == 4000)[10]) + 1          # a block boundary
    # huge runs: the reference extends the block by the run and raises at once;
    # the fast path must neither wrap its int32 run-length scan nor write outside its row.
    # Expected errors written out (the oracle would materialise a 2^31-element list)
    huge = {
        "huge_run": (np.concatenate([[0, 2**31 - 1, 5, 4000], sym]), 2**31 - 1),
        "wrapping_runs": (np.concatenate([[0, 2**30, 0, 2**30, 5, 4000], sym]), 2**30),
        "late_huge_run": (np.concatenate([sym[:k10], [7, 0, 2**31 - 1, 4000], sym[k10:]]), 2**31),
    }
    for name, (s, n_exceeded) in huge.items():
        s = np.ascontiguousarray(s, np.int32)
        with pytest.raises(ValueError) as got:
            Z.decode(s, shape)
        assert str(got.value) == f"Block size exceeded: {n_exceeded}", name
    for name, s in bad.items():
        s = np.ascontiguousarray(s, np.int32)
        try:
            want = O.zerorun_decode(list(s), shape)
        except Exception as e:  # noqa: BLE001
            with pytest.raises(type(e)) as got:
                Z.decode(s, shape)
            if not isinstance(e, IndexError):
                assert str(got.value) == str(e), name
            continue
        assert_bits(Z.decode(s, shape), want, name)


@pytest.mark.parametrize("bs,p", [(64, 64), (16, 16), (10, 64), (0, 8), (64, 80)])
def test_zerorun_random_vs_oracle(bs, p):
    """Large random sparse streams (mixed densities, all-zero / full / alternating blocks)
    against the oracle, then the decoder's round trip."""
    from ivclab_amd.entropy import ZeroRunCoder
    rng = np.random.default_rng(bs * 100 + p)
    nblk = 30000
    x = rng.integers(-200, 201, (nblk, p)).astype(np.int32)
    dens = rng.random((nblk, 1))
    x[rng.random((nblk, p)) > dens] = 0
    x[:50] = 0
    x[50:100, :] = np.where(np.arange(p) % 2 == 0, 5, 0)
    x[100:150] = rng.integers(1, 9, (50, p))
    x4 = x.reshape(10, 30, 100, p)
    Z = ZeroRunCoder(4000, bs)
    got = Z.encode(x4)
    want = O.zerorun_encode_fast(x[:, :bs] if bs else np.zeros((nblk, 0), np.int32), 4000, bs) if bs \
        else np.full(nblk, 4000, np.int32)
    assert_bits(got, want, "encode")
    dec = Z.decode(got, (10, 30, 100))
    assert_bits(dec.reshape(nblk, bs), x[:, :bs], "round trip")


def test_zerorun_device_api_and_capacity():
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(77)
    x = rng.integers(-9, 10, (5000, 64)).astype(np.int32)
    x[rng.random(x.shape) < 0.7] = 0
    want = O.zerorun_encode_fast(x)
    blocks = torch.from_numpy(x).cuda()
    off = torch.empty(5001, dtype=torch.int64, device="cuda")
    out = torch.full((want.size,), -1, dtype=torch.int32, device="cuda")
    D.zerorun_encode(blocks, off, out)
    torch.cuda.synchronize()
    assert int(off[-1]) == want.size
    assert np.array_equal(out.cpu().numpy(), want)
    # a short buffer: only the prefix that fits is written, the length is still reported
    short = torch.full((1000,), -1, dtype=torch.int32, device="cuda")
    D.zerorun_encode(blocks, off, short)
    torch.cuda.synchronize()
    assert int(off[-1]) == want.size
    assert np.array_equal(short.cpu().numpy(), want[:1000])
    # device decode
    dec = torch.empty((5000, 64), dtype=torch.int32, device="cuda")
    err = torch.empty(3, dtype=torch.int64, device="cuda")
    D.zerorun_decode(out, 5000, dec, err)
    torch.cuda.synchronize()
    assert err.cpu().tolist() == [0, 0, 0]
    assert np.array_equal(dec.cpu().numpy(), x)


@pytest.mark.parametrize("nblk", [1, 15, 16, 17, 1023, 1024 * 16 + 5, 300001, 1500001])
def test_zerorun_device_wide_and_general(nblk):
    """The device encoder's wide path (dense, 16-B aligned 64-coefficient rows: 16 blocks per
    wave-iteration) against the oracle and an independent per-block count: ends that are not
    a multiple of 16 blocks, all-zero and zero-free blocks, truncated capacity; then the same
    blocks one int32 off a 16-B boundary (general one-block-per-wave path)."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(nblk)
    x = rng.integers(-40, 41, (nblk, 64)).astype(np.int32)
    x[rng.random((nblk, 64)) > rng.random((nblk, 1))] = 0
    x[::7] = 0                                   # all-zero blocks: EOB only
    x[3::11] = rng.integers(1, 5, (len(x[3::11]), 64))   # no zeros: 65 symbols
    want = O.zerorun_encode_fast(x)
    blocks = torch.from_numpy(x).cuda()
    off = torch.full((nblk + 1,), -7, dtype=torch.int64, device="cuda")
    out = torch.full((want.size + 3,), -1, dtype=torch.int32, device="cuda")
    D.zerorun_encode(blocks, off, out)
    torch.cuda.synchronize()
    # per-block symbol counts: nonzeros + 2 per zero run before the last nonzero + EOB
    nz = x != 0
    last = np.where(nz.any(1), 63 - np.argmax(nz[:, ::-1], axis=1), -1)
    zeros = ~nz & (np.arange(64)[None] <= last[:, None])
    starts = zeros & ~np.concatenate([np.zeros((nblk, 1), bool), zeros[:, :-1]], axis=1)
    cnt = nz.sum(1) + 2 * starts.sum(1) + 1
    o = off.cpu().numpy()
    assert np.array_equal(o, np.concatenate([[0], np.cumsum(cnt)])) and o[-1] == want.size
    got = out.cpu().numpy()
    assert np.array_equal(got[:want.size], want) and (got[want.size:] == -1).all()
    cap = want.size // 3
    short = torch.full((cap,), -1, dtype=torch.int32, device="cuda")
    D.zerorun_encode(blocks, off, short)
    torch.cuda.synchronize()
    assert int(off[-1]) == want.size
    assert np.array_equal(short.cpu().numpy(), want[:cap])
    # the same blocks one int32 off a 16-B boundary take the general path
    buf = torch.zeros(nblk * 64 + 1, dtype=torch.int32, device="cuda")
    buf[1:] = blocks.view(-1)
    off2 = torch.empty(nblk + 1, dtype=torch.int64, device="cuda")
    out2 = torch.empty(want.size, dtype=torch.int32, device="cuda")
    D.zerorun_encode(buf[1:].view(nblk, 64), off2, out2)
    torch.cuda.synchronize()
    assert torch.equal(off2, off) and np.array_equal(out2.cpu().numpy(), want)


@pytest.mark.parametrize("chunks", [None, 5])
@pytest.mark.parametrize("tier", ["int8", "some_int16", "int32_value", "int16_slots_full",
                                  "dense_groups"])
def test_zerorun_int8_handoff_tiers(tier, chunks, tune):
    """The dense-row encoder hands the coefficients from its count pass to its emission pass
    as int8, a group with a value outside int8 as int16 (side slots for 1 in 8 groups), and
    falls back to emitting from the int32 rows when a value lies outside int16 or the int16
    slots run out: every tier gives the oracle's stream and offsets, in one pass and pipelined
    over 5 chunks of groups (a later chunk's wide value sends every chunk to the fallback).
    dense_groups: groups of all-nonzero blocks and groups of 896 / 897 / 512 nonzeros (the
    limits of the sparse hand-off measured in r06, profiles/r06ac_ab_zerorun_sparse.log)."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    if chunks:     # the pipelined call (count of chunk j + 1 beside the emission of chunk j)
        tune("zr_chunks", chunks)
    nblk = 16 * 2000 + 3
    rng = np.random.default_rng(hash(tier) % 1000)
    x = rng.integers(-100, 101, (nblk, 64)).astype(np.int32)
    x[rng.random((nblk, 64)) > rng.random((nblk, 1))] = 0
    x[-1, 63] = 127
    x[-2, 0] = -128
    if tier == "some_int16":           # 60 groups with values in [128, 32767]
        g = rng.choice(nblk // 16, 60, replace=False)
        x[g * 16 + 5, 7] = 32767
        x[g * 16 + 9, 63] = -32768
        x[g * 16 + 2, 0] = 128
    elif tier == "int32_value":
        x[777, 30] = 40000
    elif tier == "int16_slots_full":   # every group wide: more than the side slots
        x[::16, 1] = 300
    elif tier == "dense_groups":       # all-nonzero groups, and groups of exactly 896 / 897 nonzeros
        g = rng.choice(nblk // 16 - 4, 80, replace=False)
        for k, gi in enumerate(g):
            blk = x[gi * 16:(gi + 1) * 16]
            blk[:] = rng.integers(1, 101, (16, 64)) * rng.choice([-1, 1], (16, 64))
            if k % 4 == 1:             # 896 nonzeros: the largest packed record
                blk.reshape(-1)[rng.choice(1024, 128, replace=False)] = 0
            elif k % 4 == 2:           # 897: one past it
                blk.reshape(-1)[rng.choice(1024, 127, replace=False)] = 0
            elif k % 4 == 3:           # 512 nonzeros: exactly the emitter's first read
                blk.reshape(-1)[rng.choice(1024, 512, replace=False)] = 0
    want = O.zerorun_encode_fast(x)
    blocks = torch.from_numpy(x).cuda()
    off = torch.full((nblk + 1,), -7, dtype=torch.int64, device="cuda")
    out = torch.full((want.size + 2,), -1, dtype=torch.int32, device="cuda")
    D.zerorun_encode(blocks, off, out)
    torch.cuda.synchronize()
    o = off.cpu().numpy()
    assert o[-1] == want.size
    got = out.cpu().numpy()
    assert np.array_equal(got[:want.size], want) and (got[want.size:] == -1).all()
    # offsets: every block's slice ends with its EOB and holds its symbol count
    nz = x != 0
    last = np.where(nz.any(1), 63 - np.argmax(nz[:, ::-1], axis=1), -1)
    zeros = ~nz & (np.arange(64)[None] <= last[:, None])
    starts = zeros & ~np.concatenate([np.zeros((nblk, 1), bool), zeros[:, :-1]], axis=1)
    cnt = nz.sum(1) + 2 * starts.sum(1) + 1
    assert np.array_equal(o, np.concatenate([[0], np.cumsum(cnt)]))
    assert (got[o[1:] - 1] == 4000).all()


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_zerorun_device_unaligned_stream(shift):
    """The wide path's 16-byte stream stores when the caller's output starts 4, 8 or 12 bytes
    past a 16-byte boundary (a view into a larger buffer), with a capacity that cuts a quad."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    nblk = 1024 * 16 + 5
    rng = np.random.default_rng(100 + shift)
    x = rng.integers(-40, 41, (nblk, 64)).astype(np.int32)
    x[rng.random((nblk, 64)) > rng.random((nblk, 1))] = 0
    want = O.zerorun_encode_fast(x)
    blocks = torch.from_numpy(x).cuda()
    off = torch.empty(nblk + 1, dtype=torch.int64, device="cuda")
    buf = torch.full((want.size + 8,), -1, dtype=torch.int32, device="cuda")
    D.zerorun_encode(blocks, off, buf[shift:shift + want.size])
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    assert (got[:shift] == -1).all() and (got[shift + want.size:] == -1).all()
    assert np.array_equal(got[shift:shift + want.size], want)
    cap = want.size // 2 + 1
    buf.fill_(-1)
    D.zerorun_encode(blocks, off, buf[shift:shift + cap])
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    assert int(off[-1]) == want.size
    assert np.array_equal(got[shift:shift + cap], want[:cap]) and (got[shift + cap:] == -1).all()


def test_zerorun_after_fused_intra():
    """The codec chain: fused intra encode with zig-zag -> zero-run stream -> decode ->
    back to the quantised blocks, against the oracle's chain."""
    from ivclab_amd.entropy import ZeroRunCoder
    N, L = _native()
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (1, 64, 96, 1), dtype=np.uint8)
    img[0, :24] = 128
    t = N.table_arg(PatchQuant(0.5).get_quantization_table())
    zz = np.empty((8, 12, 3, 64), np.int32)
    N.check(L.ivc_intra_encode(N.ptr(img), 1, 1, 64, 96, 1, N.ptr(t), N.F64, 1, N.ptr(zz)))
    want_zz = O.intra_encode(img[0], 0.5, zigzag=True)
    assert_bits(zz, want_zz, "zig-zag")
    sym = ZeroRunCoder().encode(zz)
    assert_bits(sym, O.zerorun_encode(want_zz), "stream")
    assert_bits(ZeroRunCoder().decode(sym, (8, 12, 3)), want_zz, "decoded")


def test_minmax_host_and_device():
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    N, L = _native()
    rng = np.random.default_rng(8)
    for n in (0, 1, 7, 100003):
        x = rng.integers(-(1 << 31), (1 << 31) - 1, n, dtype=np.int64).astype(np.int32)
        mm = np.zeros(2, np.int32)
        N.check(L.ivc_minmax_i32(N.ptr(x), n, N.ptr(mm)))
        want = [x.min(), x.max()] if n else [np.iinfo(np.int32).max, np.iinfo(np.int32).min]
        assert mm.tolist() == list(map(int, want))
        t = torch.from_numpy(x).cuda()
        dm = torch.zeros(2, dtype=torch.int32, device="cuda")
        D.minmax(t, dm)
        assert dm.cpu().tolist() == list(map(int, want))
    # views starting off 16 B, lengths around the vector/unroll edges, extremes in the head,
    # the body and the tail
    base = rng.integers(-1000, 1000, (1 << 20) + 11).astype(np.int32)
    tb = torch.from_numpy(base).cuda()
    for off in (0, 1, 2, 3):
        for n in (1, 3, 4, 5, 17, 4099, 1 << 16, (1 << 20) + 11 - off):
            for pos in (0, n // 2, n - 1):
                v = base[off:off + n].copy()
                v[pos] = -5000 if pos != n - 1 else 5000
                tb[off:off + n] = torch.from_numpy(v).cuda()
                dm = torch.zeros(2, dtype=torch.int32, device="cuda")
                D.minmax(tb[off:off + n], dm)
                assert dm.cpu().tolist() == [int(v.min()), int(v.max())], (off, n, pos)
                tb[off:off + n] = torch.from_numpy(base[off:off + n]).cuda()


def _zr_chain(img, table, scale=None):
    """Oracle chain: per frame zero-run(zig-zag(quantize(dct(patch)))) concatenated."""
    out = []
    for f in range(img.shape[0]):
        d = O.dct_transform(O.patch(img[f]))
        q = np.round(d / table[None, None]).astype(np.int32)
        out.append(O.zerorun_encode_fast(O.zigzag_flatten(q)))
    return np.concatenate(out) if out else np.zeros(0, np.int32)


@pytest.mark.parametrize("case", ["s1", "s05", "s007", "s0005", "custom", "rgb", "ragged"])
def test_intra_symbols_fused_vs_oracle(case):
    """Pixels -> zero-run symbols (count pass, scan, emitter from the count pass's int8 hand-off)
    against the oracle's per-op chain.  s007: groups with values outside int8 (the int16 slot);
    s0005: values outside int16, where the emitter stands down and the fused emission pass
    (which redoes the transform) runs."""
    N, L = _native()
    rng = np.random.default_rng(hash(case) % 1000)
    F, H, W, C = 2, 48, 128, 1
    scale = {"s1": 1.0, "s05": 0.5, "s007": 0.07, "s0005": 0.0005}.get(case, 1.0)
    if case == "rgb":
        C = 3
    if case == "ragged":
        W = 264                                     # 33 blocks: the last group holds 1 block
    img = rng.integers(0, 256, (F, H, W, C), dtype=np.uint8)
    img[:, :16] = img[:, :1, :1]                    # flat blocks: all-zero AC, EOB-only planes
    img[:, 16:24] = np.arange(W, dtype=np.uint8)[None, None, :, None] // 3
    table = PatchQuant(scale).get_quantization_table().astype(np.float64)
    if case == "custom":
        table[2] *= 1.61                            # planes 1 and 2 differ
    want = _zr_chain(img, table)
    cap = want.size + 5
    out = np.full(cap, -7, np.int32)
    nsym = np.zeros(1, np.int64)
    N.check(L.ivc_intra_symbols(N.ptr(img), 1, F, H, W, C, N.ptr(N.table_arg(table)), 4000,
                                N.ptr(out), cap, N.ptr(nsym)))
    assert int(nsym[0]) == want.size
    assert_bits(out[:want.size], want, case)
    # too small a buffer: an error that reports the needed length
    with pytest.raises(ValueError):
        N.check(L.ivc_intra_symbols(N.ptr(img), 1, F, H, W, C, N.ptr(N.table_arg(table)), 4000,
                                    N.ptr(out), want.size - 1, N.ptr(nsym)))
    assert int(nsym[0]) == want.size


def test_intra_symbols_device_and_4k():
    """Device API on a full 4K luma frame pair, and a capacity-limited prefix."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(4096)
    img = rng.integers(0, 256, (2, 2160, 3840), dtype=np.uint8)
    img[0, :800] = 90
    table = PatchQuant(1.0).get_quantization_table()
    want = _zr_chain(img[..., None], table.astype(np.float64))
    fr = torch.from_numpy(img).cuda()
    nsym = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty(want.size, dtype=torch.int32, device="cuda")
    D.intra_symbols(fr, table, out, nsym)
    torch.cuda.synchronize()
    assert int(nsym.item()) == want.size
    assert np.array_equal(out.cpu().numpy(), want)
    short = torch.full((12345,), -1, dtype=torch.int32, device="cuda")
    D.intra_symbols(fr, table, short, nsym)
    torch.cuda.synchronize()
    assert int(nsym.item()) == want.size
    assert np.array_equal(short.cpu().numpy(), want[:12345])


@pytest.mark.parametrize("case", ["s1", "s007", "s0005", "custom", "rgb", "ragged"])
def test_intra_symbols_emission_histogram(case):
    """The emission pass's clamped histogram of the stream (ivc_intra_symbols_hist_dev) equals
    the oracle's histogram of the oracle stream: a wide guarded range (values past +-512 take
    the global path at scale 0.07), a narrow one (most symbols, EOB included, clamp into the end
    bins), accumulation onto existing counts, and a capacity-cut stream (counted whole)."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(len(case) * 7 + 3)
    F, H, W, C = 2, 48, 136, 1
    scale = {"s1": 1.0, "s007": 0.07, "s0005": 0.0005}.get(case, 0.5)
    if case == "rgb":
        C = 3
    if case == "ragged":
        W = 264
    img = rng.integers(0, 256, (F, H, W, C), dtype=np.uint8)
    img[:, :16] = img[:, :1, :1]
    table = PatchQuant(scale).get_quantization_table().astype(np.float64)
    if case == "custom":
        table[2] *= 1.61
    want = _zr_chain(img, table)
    fr = torch.from_numpy(img if C == 3 else img[..., 0]).cuda()
    nsym = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.empty(want.size, dtype=torch.int32, device="cuda")
    for lo, n in [(-4097, 8194), (-3, 9)]:
        hist = torch.zeros(n, dtype=torch.int64, device="cuda")
        D.intra_symbols(fr, table, out, nsym, hist=hist, hist_lo=lo)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)
        ref = O.histogram(want, lo, n)
        assert np.array_equal(hist.cpu().numpy(), ref), (case, lo, n)
        if lo == -3:
            D.intra_symbols(fr, table, out[:want.size // 3], nsym, hist=hist, hist_lo=lo)
            torch.cuda.synchronize()
            assert np.array_equal(hist.cpu().numpy(), 2 * ref), "accumulated / capacity-cut"
    if case == "s007":                              # the out-of-LDS-range path ran
        assert (np.abs(want[want != 4000]) >= 512).any()


@pytest.mark.parametrize("case,chunks", [("s1", 2), ("s1", 5), ("s007", 3), ("s0005", 2),
                                        ("rgb", 4), ("ragged", 5), ("odd_rows", 3)])
def test_intra_symbols_pipelined_chunks(tune, case, chunks):
    """The count pass and the emitter pipelined over chunks of whole frames
    (the sym_chunks override; the bench's 256 x 4K call takes 16): stream, length and emission
    histogram equal the oracle's for every hand-off tier (s007: int16 slots; s0005: the
    emitters stand down and the fused emission pass runs over every frame), a capacity-cut
    stream, and a frame whose group count is not a multiple of 4 (odd_rows: one chunk)."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    tune("sym_chunks", chunks)
    rng = np.random.default_rng(chunks * 31 + len(case))
    F, H, W, C = 5, 48, 128, 1
    scale = {"s007": 0.07, "s0005": 0.0005}.get(case, 1.0)
    if case == "rgb":
        C = 3
    if case == "ragged":
        W = 264                                     # 33 blocks: the last group holds 1 block
    if case == "odd_rows":
        H = 40                                      # 5 block rows: 10 groups per frame
    img = rng.integers(0, 256, (F, H, W, C), dtype=np.uint8)
    img[:, :16] = img[:, :1, :1]
    img[2] = 128                                    # a flat frame inside a chunk
    table = PatchQuant(scale).get_quantization_table().astype(np.float64)
    want = _zr_chain(img, table)
    fr = torch.from_numpy(img if C == 3 else img[..., 0]).cuda()
    nsym = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.full((want.size,), -1, dtype=torch.int32, device="cuda")
    hist = torch.zeros(8194, dtype=torch.int64, device="cuda")
    D.intra_symbols(fr, table, out, nsym, hist=hist, hist_lo=-4097)
    torch.cuda.synchronize()
    assert int(nsym.item()) == want.size
    assert_bits(out.cpu().numpy(), want, (case, chunks))
    assert np.array_equal(hist.cpu().numpy(), O.histogram(want, -4097, 8194)), (case, chunks)
    cut = torch.full((want.size // 3,), -1, dtype=torch.int32, device="cuda")
    D.intra_symbols(fr, table, cut, nsym)
    torch.cuda.synchronize()
    assert int(nsym.item()) == want.size
    assert np.array_equal(cut.cpu().numpy(), want[:want.size // 3])


@pytest.mark.parametrize("chunks", [2, 5])
def test_intra_symbols_pipelined_late_int16_overflow(tune, chunks):
    """Only the LAST frame holds a coefficient outside int16, so only the last chunk's count pass
    sets the stand-down word: the emitters of the earlier chunks may already have run (and
    counted their symbols) when it is set.  The emission histogram must still count every symbol
    exactly once (the emitters' counts join the caller's histogram only when no chunk stood
    down), and the stream must equal the oracle's."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    tune("sym_chunks", chunks)
    rng = np.random.default_rng(chunks)
    F, H, W = 5, 48, 128
    img = rng.integers(0, 3, (F, H, W, 1), dtype=np.uint8)       # dim frames: |coef| <= int16
    img[-1] = rng.integers(0, 256, (H, W, 1), dtype=np.uint8)    # the bright last frame
    table = PatchQuant(0.0005).get_quantization_table().astype(np.float64)
    peak = [np.abs(np.round(O.dct_transform(O.patch(img[f])) / table[None, None])).max() for f in range(F)]
    assert max(peak[:-1]) <= 32767 < peak[-1], peak
    want = _zr_chain(img, table)
    fr = torch.from_numpy(img[..., 0]).cuda()
    nsym = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = torch.full((want.size,), -1, dtype=torch.int32, device="cuda")
    ref = O.histogram(want, -4097, 8194)
    for rep in range(3):
        hist = torch.zeros(8194, dtype=torch.int64, device="cuda")
        D.intra_symbols(fr, table, out, nsym, hist=hist, hist_lo=-4097)
        torch.cuda.synchronize()
        assert int(nsym.item()) == want.size
        assert_bits(out.cpu().numpy(), want, (chunks, rep))
        assert np.array_equal(hist.cpu().numpy(), ref), (chunks, rep)


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_intra_symbols_unaligned_stream(shift):
    """The fused emit's 16-byte stores when the output view starts 4/8/12 bytes past a 16-byte
    boundary, whole and capacity-cut in the middle of a quad."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(shift)
    img = rng.integers(0, 256, (1, 272, 480), dtype=np.uint8)
    img[0, :64, :128] = 77
    table = PatchQuant(0.5).get_quantization_table()
    want = _zr_chain(img[..., None], table.astype(np.float64))
    fr = torch.from_numpy(img).cuda()
    nsym = torch.zeros(1, dtype=torch.int64, device="cuda")
    buf = torch.full((want.size + 8,), -1, dtype=torch.int32, device="cuda")
    D.intra_symbols(fr, table, buf[shift:shift + want.size], nsym)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    assert int(nsym.item()) == want.size
    assert np.array_equal(got[shift:shift + want.size], want)
    assert (got[:shift] == -1).all() and (got[shift + want.size:] == -1).all()
    cap = want.size // 2 + 1
    buf.fill_(-1)
    D.intra_symbols(fr, table, buf[shift:shift + cap], nsym)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    assert np.array_equal(got[shift:shift + cap], want[:cap]) and (got[shift + cap:] == -1).all()


# ------------------------------------------------------------------------- colour ------
def test_color_golden_gpu(golden):
    from ivclab_amd.signal.color import rgb2gray, rgb2ycbcr, ycbcr2rgb
    c = golden("color")
    for k in ("rgb_u8", "rgb_f64", "rgb_f32", "rgb_i16"):
        assert_bits(rgb2ycbcr(c[k]), c[f"{k}_ycc"], k)
    for k in ("rgb_u8", "rgb_f64", "rgb_f32"):
        assert_bits(rgb2gray(c[k]), c[f"{k}_gray"], k)
    for k in ("ycc_f64", "ycc_f32", "ycc_u8", "ycc4_f64"):
        assert_bits(ycbcr2rgb(c[k]), c[f"{k}_rgb"], k)
    assert_bits(ycbcr2rgb(rgb2ycbcr(c["rgb_u8"])), c["round_trip"], "round trip")


def test_color_large_vs_oracle():
    """1080p frames: the elementwise conversions against NumPy itself, rgb2ycbcr against the
    exact k-order-FMA restatement on a pixel sample (NumPy's own matmul depends on the host
    BLAS kernel; the fixtures pin it where they were made)."""
    from ivclab_amd.signal.color import rgb2gray, rgb2ycbcr, ycbcr2rgb
    rng = np.random.default_rng(1080)
    img = rng.integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
    ycc = rgb2ycbcr(img)
    idx = rng.integers(0, 1080 * 1920, 1500)
    want = O.rgb2ycbcr_fma(img.reshape(-1, 3)[idx][:, None, :])[:, 0, :]
    assert_bits(ycc.reshape(-1, 3)[idx], want, "rgb2ycbcr sample")
    assert_bits(ycbcr2rgb(ycc), O.ycbcr2rgb(ycc), "ycbcr2rgb")
    assert_bits(rgb2gray(img), O.rgb2gray(img), "rgb2gray")
    f = rng.normal(100, 80, (64, 64, 3)).astype(np.float32)
    assert_bits(ycbcr2rgb(f), O.ycbcr2rgb(f), "f32")
    assert_bits(rgb2gray(f), O.rgb2gray(f), "f32 gray")
    with pytest.raises(ValueError):
        rgb2ycbcr(np.zeros((4, 4, 2)))


# ---------------------------------------------------------------------- IntraCodec -----
def _chain_symbols(ycc, scale):
    """Oracle: image2symbols (intracodec.py:66-81) from an already colour-converted image."""
    if ycc.ndim == 2:
        ycc = ycc[:, :, None]
    H, W, _ = ycc.shape
    ph, pw = (8 - H % 8) % 8, (8 - W % 8) % 8
    if ph or pw:
        ycc = np.pad(ycc, ((0, ph), (0, pw), (0, 0)), mode="edge")
    q = O.quantize(O.dct_transform(O.patch(ycc)), scale)
    return O.zerorun_encode(O.zigzag_flatten(q))


def _chain_image(sym, shape, scale):
    """Oracle: symbols2image (intracodec.py:93-146)."""
    if len(shape) == 2:
        (H, W), C, rgb = shape, 1, False
    else:
        (H, W, C), rgb = shape, True
    dec = O.zerorun_decode(sym, (H // 8, W // 8, C))
    rec = O.unpatch(O.dct_inverse(O.dequantize(O.zigzag_unflatten(dec), scale)))
    rec = rec[:H, :W, :]
    if C == 1:
        return rec[:, :, 0] if rec.shape[2] == 1 else rec
    return O.ycbcr2rgb(rec) if rgb else rec


@pytest.mark.parametrize("case", ["gray_u8", "gray_u8_pad", "gray_f64", "rgb_u8", "ycc_u8"])
def test_intracodec_symbols_and_image(golden, case):
    from ivclab_amd.image import IntraCodec
    rng = np.random.default_rng(len(case))
    scale = 0.6
    codec = IntraCodec(quantization_scale=scale)
    if case == "rgb_u8":
        c = golden("color")
        img, ycc, rgb = c["rgb_u8"], c["rgb_u8_ycc"], True
    else:
        shape = {"gray_u8": (64, 80), "gray_u8_pad": (50, 70), "gray_f64": (48, 56),
                 "ycc_u8": (40, 48, 3)}[case]
        img = rng.integers(0, 256, shape).astype(np.float64 if case == "gray_f64" else np.uint8)
        if case == "gray_f64":
            img = img + rng.random(shape)
        ycc, rgb = img, False
    sym = codec.image2symbols(img, is_source_rgb=rgb)
    assert_bits(sym, _chain_symbols(ycc, scale), "image2symbols")
    out_shape = img.shape
    assert_bits(codec.symbols2image(sym, out_shape), _chain_image(sym, out_shape, scale),
                "symbols2image")


@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("zz", [0, 1])
@pytest.mark.parametrize("rgb", [0, 1])
def test_intra_decode_image_vs_oracle(C, zz, rgb):
    """ivc_intra_decode_image (the decode chain with the unpatch fused, ivc_decode.hip):
    unflatten -> dequantise (C = 1 broadcast over 3 planes) -> IDCT -> unpatch (-> ycbcr2rgb)
    against the oracle on 2 frames of 24 x 152 (19 block columns: ragged 8-block groups),
    coefficients from quantised content, extremes whose dequantised value overflows int32
    (INT32_MIN, as x86 NumPy casts) and scales down to 0.013."""
    N, L = _native()
    rng = np.random.default_rng(100 * C + 10 * zz + rgb)
    F, H, W = 2, 24, 152
    for scale in (1.0, 0.013, 2.5):
        q = rng.integers(-60, 61, (F, H // 8, W // 8, C, 64)).astype(np.int32)
        q[..., 0] = rng.integers(-1000, 1000, q.shape[:-1])
        q[0, 0, 0] = np.iinfo(np.int32).max                       # dequantise overflows
        q[1, 1, 3] = np.iinfo(np.int32).min
        q[0, 2, 18, 0, 5] = 0
        table = PatchQuant(scale).get_quantization_table()
        t = N.table_arg(table)
        out = np.full((F, H, W, 3), np.nan)
        N.check(L.ivc_intra_decode_image(N.ptr(q), F, H, W, C, N.ptr(t), zz, rgb, N.ptr(out)))
        for f in range(F):
            qf = q[f] if zz else q[f].reshape(q[f].shape[:-1] + (8, 8))
            want = O.unpatch(O.intra_decode(qf, scale, unzigzag=bool(zz)))
            if rgb:
                want = O.ycbcr2rgb(want)
            assert_bits(out[f], want, f"decode image C={C} zz={zz} rgb={rgb} scale={scale} f={f}")
    assert L.ivc_intra_decode_image(N.ptr(q), F, H, W, 2, N.ptr(t), zz, rgb, N.ptr(out)) == N.E_SHAPE
    assert L.ivc_intra_decode_image(N.ptr(q), F, H, 12, C, N.ptr(t), zz, rgb, N.ptr(out)) == N.E_SHAPE


def test_symbols2image_stream_errors_match_reference():
    """IntraCodec.symbols2image on the device raises what the reference's chain raises for a
    malformed stream (ZeroRunCoder.decode, zerorun.py:46-88): a block overflowing 64, a
    stream ending inside a block, right after a zero, or with too few blocks; trailing symbols
    after the last expected block are ignored."""
    from ivclab_amd.image import IntraCodec
    codec = IntraCodec(quantization_scale=1.0)
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (16, 24)).astype(np.uint8)
    sym = np.asarray(codec.image2symbols(img, is_source_rgb=False))
    shape = (16, 24, 3)
    good = codec.symbols2image(sym, shape)
    assert_bits(good, _chain_image(sym, shape, 1.0), "clean stream")
    assert_bits(codec.symbols2image(np.concatenate([sym, [0, 0, 7]]).astype(np.int32), shape), good,
                "trailing symbols ignored")
    bad = {
        "overflow": np.concatenate([[0, 70], sym]).astype(np.int64),
        "ends_inside": sym[:-1],
        "ends_after_zero": np.array([3, 0]),
        "too_few": sym[: np.flatnonzero(sym == 4000)[2] + 1],
    }
    for name, s in bad.items():
        with pytest.raises(Exception) as got:
            codec.symbols2image(s, shape)
        with pytest.raises(Exception) as want:
            O.zerorun_decode(list(s), (2, 3, 3))
        assert type(got.value) is type(want.value), (name, got.value, want.value)
        if not isinstance(want.value, IndexError):
            assert str(got.value) == str(want.value), name


def test_intracodec_encode_decode_roundtrip():
    """Huffman-coded round trip: the decoded image is symbols2image(image2symbols(img)) and
    the bit count is the sum of the symbols' code lengths."""
    from ivclab_amd.image import IntraCodec
    rng = np.random.default_rng(11)
    img = rng.integers(0, 256, (64, 96, 3)).astype(np.uint8)
    img[:32] = 128
    codec = IntraCodec(quantization_scale=1.0)
    codec.train_huffman_from_image(img)
    rec, bitstream, bitsize, bpp = codec.encode_decode(img, return_bpp=True)
    sym = codec.image2symbols(img)
    assert np.array_equal(rec, codec.symbols2image(sym, img.shape))
    L = codec.huffman.encoder_codebook
    assert bitsize == float(L[sym - codec.bounds[0]].astype(np.int64).sum())
    assert bpp == bitsize / (64 * 96)
    assert codec.huffman.is_prefix_free()
    bs, _ = codec.intra_encode(img)
    assert np.array_equal(codec.intra_decode(bs, img.shape), rec)


def test_videocodec_iframe_and_pframe():
    """VideoCodec (videocodec.py:37-86): frame 0 is the oracle chain on the luma plane
    (rgb2ycbcr of the float32 frame, the 3-plane quantisation of a grayscale input, the
    first plane of the 3-channel reconstruction clipped into Y, ycbcr2rgb, uint8); its bit
    count is the Huffman code lengths of the frame's symbols.  Frame 1 raises ValueError as
    the reference does: the motion-vector coder trained on [-40, 40] meets indices up to 80."""
    from ivclab_amd.video import VideoCodec
    rng = np.random.default_rng(31)
    scale = 0.8
    frame = rng.integers(0, 256, (32, 48, 3)).astype(np.uint8)
    codec = VideoCodec(quantization_scale=scale)
    rec, bitstream, bits = codec.encode_decode(frame, frame_num=0)
    ycc = O.rgb2ycbcr_fma(frame.astype(np.float32))
    y = ycc[..., 0]
    sym = _chain_symbols(y, scale)
    rec_y = _chain_image(sym, y.shape, scale)
    assert rec_y.shape == (32, 48, 3) and codec.decoder_recon.shape == (32, 48, 3)
    assert_bits(codec.decoder_recon, rec_y, "I-frame luma reconstruction")
    want = ycc.copy()
    want[..., 0] = np.clip(rec_y[..., 0], 0, 255)
    assert_bits(rec, O.ycbcr2rgb(want).astype(np.uint8), "I-frame RGB")
    L = codec.intra_codec.huffman.encoder_codebook
    assert bits == float(L[sym - codec.intra_codec.bounds[0]].astype(np.int64).sum())
    nxt = np.roll(frame, (2, -3), axis=(0, 1))
    mv = O.motion_vectors(codec.decoder_recon[..., 0], O.rgb2ycbcr_fma(nxt.astype(np.float32))[..., 0], 4)
    assert mv.max() > 40
    with pytest.raises(ValueError, match="outside the trained range"):
        codec.encode_decode(nxt, frame_num=1)


def test_stats_marg_gpu_vs_oracle():
    """stats_marg on the GPU histogram equals np.histogram's counts (dropped out-of-range
    values, closed last bin) divided by the sample count."""
    from ivclab_amd.entropy import stats_marg
    rng = np.random.default_rng(21)
    for dt in (np.uint8, np.int16, np.int32, np.int64):
        x = rng.integers(-300 if dt != np.uint8 else 0, 256, (50, 60)).astype(dt)
        for edges in (np.arange(256), np.arange(-20, 41), np.arange(10, 12)):
            assert_bits(stats_marg(x, edges), O.stats_marg(x, edges), f"{dt} {edges[0]}")
    # 64-bit and unsigned 32-bit data stay on the integer kernels (int64 path) while the edges
    # lie inside +-2^53: values beyond 2^53 / 2^63, and edges near +-2^52 and past int32
    big = np.array([0, 5, -7, 1 << 53, (1 << 53) + 1, -(1 << 60), np.iinfo(np.int64).max,
                    np.iinfo(np.int64).min, (1 << 52) - 1, -(1 << 52), 3_000_000_000], np.int64)
    for edges in (np.arange(-8, 9), np.arange((1 << 52) - 3, (1 << 52) + 2),
                  np.arange(-(1 << 52) - 2, -(1 << 52) + 3), np.arange(2_999_999_998, 3_000_000_003)):
        assert_bits(stats_marg(big, edges), O.stats_marg(big, edges), f"int64 {edges[0]}")
    u = np.array([0, 1, 7, 1 << 63, (1 << 64) - 1, 4_000_000_000], np.uint64)
    for edges in (np.arange(0, 9), np.arange(3_999_999_998, 4_000_000_002)):
        assert_bits(stats_marg(u, edges), O.stats_marg(u, edges), f"uint64 {edges[0]}")
        u32 = np.array([0, 1, 7, 3_999_999_999, 4_000_000_000, (1 << 32) - 1], np.uint32)
        assert_bits(stats_marg(u32, edges), O.stats_marg(u32, edges), f"uint32 {edges[0]}")


STATS = ["u8_full", "i16_window", "i64_unit", "f64_linspace", "f32_nonuniform", "f64_intbins",
         "f64_edges_special", "f64_inf_edges", "u8_float_edges", "u8_step_edges"]


@pytest.mark.parametrize("case", STATS)
def test_stats_marg_golden_gpu(golden, case):
    """The GPU stats_marg (integer kernel for small-integer data over unit edges, the edge
    kernel for everything else) against the reference's own pmf, bit for bit."""
    from ivclab_amd.entropy import calc_entropy, smooth_pmf, stats_marg
    s = golden("stats")
    x, bins = s[f"{case}_x"], s[f"{case}_bins"]
    bins = int(bins) if bins.ndim == 0 else bins
    pmf = stats_marg(x, bins)
    assert_bits(pmf, s[f"{case}_pmf"], case)
    assert_bits(smooth_pmf(pmf), s[f"{case}_smooth"], case)
    assert_bits(np.float64(calc_entropy(pmf)), s[f"{case}_entropy"], case)


def test_stats_marg_edge_kernel_large_and_errors():
    """The edge kernel past its LDS capacity (5000 edges: global path), on 2M non-integer
    samples, and np.histogram's errors (decreasing edges, a non-finite autodetected range)."""
    from ivclab_amd.entropy import stats_marg
    rng = np.random.default_rng(5)
    x = rng.normal(0, 40, (1000, 2000))
    x[::97, ::13] = np.nan
    for edges in (np.linspace(-100, 100, 5000), np.sort(rng.normal(0, 50, 300)), np.array([0.0, 0.0, 1.0])):
        assert_bits(stats_marg(x, edges), O.stats_marg(x, edges), f"{edges.size} edges")
    assert_bits(stats_marg(x[1:8].astype(np.float32), 33), O.stats_marg(x[1:8].astype(np.float32), 33))
    with pytest.raises(ValueError):
        stats_marg(x, np.array([3.0, 2.0, 1.0]))
    with pytest.raises(ValueError):
        stats_marg(np.array([1.0, np.nan]), 4)


@pytest.mark.parametrize("sr", [4, 8, 16])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_me_float_search_kernel(sr, dtype):
    """The LDS-window float search (me_flt_kernel, sr in {4, 8, 16}) against the C oracle's
    NumPy-order SSD: non-integer frames with a shift, an 8-periodic reference (every candidate
    has the same multiset of squares: the winner is decided by the rounding order), flat ties,
    NaN / inf pixels, and frame sizes narrower / not a multiple of a workgroup round."""
    rng = np.random.default_rng(sr * 7 + np.dtype(dtype).itemsize)
    for H, W in ((16, 16), (8, 224), (72, 264), (136, 120), (48, 8)):
        a = rng.normal(128, 50, (H + 40, W + 40)).astype(dtype)
        ref, cur = a[:H, :W].copy(), (a[3:H + 3, 5:W + 5] + rng.normal(0, 0.3, (H, W))).astype(dtype)
        tile = rng.normal(100, 30, (8, 8))
        per = np.tile(tile, (H // 8 + 1, W // 8 + 1))[:H, :W].astype(dtype)
        cur_p = np.roll(per, (1, 2), axis=(0, 1)) + dtype(0.37)
        nan_ref = ref.copy()
        nan_ref[::9, ::11] = np.nan
        nan_ref[5, :] = np.inf
        flat = np.full((H, W), 3.25, dtype)
        for r_, c_, what in ((ref, cur, "shift"), (per, cur_p, "periodic"), (nan_ref, cur, "nan/inf"),
                             (flat, flat, "flat"), (cur, np.full((H, W), np.nan, dtype), "all-nan")):
            mv = MotionCompensator(sr).compute_motion_vector(r_, c_)
            assert_bits(mv, c_motion_vectors(r_, c_, sr), f"{np.dtype(dtype).name} sr={sr} {H}x{W} {what}")


def _pairwise_ssd_all(ref, cur, sr, by, bx):
    """Every in-frame candidate's float64 SSD of block (by, bx) in NumPy's order (the
    reference's np.sum over the 64 squares), as {raster index: value}."""
    n, (H, W) = 2 * sr + 1, ref.shape
    blk = cur[8 * by:8 * by + 8, 8 * bx:8 * bx + 8]
    out = {}
    for dy in range(-sr, sr + 1):
        for dx in range(-sr, sr + 1):
            y, x = 8 * by + dy, 8 * bx + dx
            if 0 <= y <= H - 8 and 0 <= x <= W - 8:
                out[(dy + sr) * n + dx + sr] = np.sum((ref[y:y + 8, x:x + 8] - blk) ** 2)
    return out


def _near_tie_pair(rng, H, W):
    """Two independent frames of two grey levels mapped through the luma scale of VideoCodec's
    float64 luma (y = k * 219/255 + 16): every nonzero difference is the same value, so
    candidates with equal mismatch counts have float64 SSDs that differ only by how the
    pairwise order rounds their column sums — exact ties and ulp-level near ties at the
    minimum, which only the exact phase can order."""
    ref = rng.integers(0, 2, (H, W)) * (219.0 / 255.0) + 16.0
    cur = rng.integers(0, 2, (H, W)) * (219.0 / 255.0) + 16.0
    return ref, cur


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_me_f64_pruned_search_exact(mode, tune):
    """The float64 search with its float32 bound phase (mode 0, the default), without it (1) and
    with every round deferred to the float64 kernel (2) against the C oracle (NumPy-order SSD,
    first strict minimum): ulp-level near ties (checked to exist: blocks whose best and
    runner-up float64 SSDs differ by one to a few ulps), an 8-periodic reference (same squares
    in every candidate: order decides), a half-flat frame (its rounds overflow the candidate
    list and are deferred, the others are not), values past 2^24 and below 2^-60 in a few rounds
    (the bound's assumptions fail: deferred), NaN and inf pixels, and a frame narrower than a
    round, at sr = 4, 8 and 16."""
    tune("f64_me", mode)
    rng = np.random.default_rng(640 + mode)
    ref, cur = _near_tie_pair(rng, 48, 200)
    close = ties = 0
    for by in range(6):
        for bx in range(25):
            v = np.array(sorted(_pairwise_ssd_all(ref, cur, 16, by, bx).values()))
            close += int(0 < v[1] - v[0] <= 4 * np.spacing(v[1]))
            ties += int(v[1] == v[0])
    assert close >= 4 and ties >= 10, ("the fixture lacks near ties at the minimum", close, ties)
    H, W = 72, 264
    a = rng.normal(128, 50, (H + 40, W + 40))
    r1, c1 = a[:H, :W].copy(), a[3:H + 3, 5:W + 5] + rng.normal(0, 0.3, (H, W))
    tile = rng.normal(100, 30, (8, 8))
    per = np.tile(tile, (H // 8 + 1, W // 8 + 1))[:H, :W]
    cur_p = np.roll(per, (1, 2), axis=(0, 1)) + 0.37
    half = r1.copy(); halfc = c1.copy()
    half[:, :120] = 16.0; halfc[:, :120] = 16.0                 # letterbox-like flat left part
    big, tiny = r1.copy(), c1.copy()
    big[8:16, 200:208] *= 2.0 ** 20                              # > 2^24 in one round
    tiny[40:48, 16:24] = 1e-30                                   # < 2^-60 in another
    nan = r1.copy()
    nan[::9, ::11] = np.nan
    nan[5, :] = np.inf
    cases = [(ref, cur, "near ties"), (per, cur_p, "periodic"), (half, halfc, "half flat"),
             (big, c1, "big"), (r1, tiny, "tiny"), (nan, c1, "nan/inf"),
             (r1[:, :40].copy(), c1[:, :40].copy(), "narrow")]
    for sr in (4, 8, 16):
        for r_, c_, what in cases:
            mv = MotionCompensator(sr).compute_motion_vector(r_, c_)
            assert_bits(mv, c_motion_vectors(r_, c_, sr), f"mode {mode} sr={sr} {what}")


def test_me_float_search_device_frames_and_1080p():
    """Several frame pairs in one device call (rounds over frames), and a full non-integer
    1080p float64 pair at sr = 16 checked on sampled block rows."""
    import torch
    import ivclab_amd.device as D
    rng = np.random.default_rng(1920)
    lo = rng.normal(120, 40, (290, 500))
    big = np.kron(lo, np.ones((4, 4)))[:1120, :1960] * (219 / 255) + 16.0 + rng.normal(0, 1.5, (1120, 1960))
    fr = np.stack([big[k:k + 1080, 2 * k:2 * k + 1920] for k in range(3)])
    t = torch.from_numpy(np.ascontiguousarray(fr)).cuda()
    mv = torch.empty((2, 135, 240), dtype=torch.int64, device="cuda")
    D.motion_estimate(t[:-1].contiguous(), t[1:].contiguous(), 16, mv)
    got = mv.cpu().numpy()
    for p in range(2):
        for rows in ((0, 3), (67, 70), (132, 135)):
            want = c_motion_vectors(fr[p], fr[p + 1], 16, rows=rows)[..., 0]
            assert_bits(got[p, rows[0]:rows[1]], want, f"pair {p} rows {rows}")


@pytest.mark.parametrize("zz", [0, 1])
@pytest.mark.parametrize("case", ["jpeg", "fine", "custom"])
def test_inter_encode_encoder_histogram(zz, case):
    """ivc_inter_encode_hist_dev (the residual encoder accumulating its output's histogram,
    OUT_COEFH; ivclab/entropy/entropy.py:6-29 over VideoCodec's residual coefficients): the
    output equals ivc_inter_encode_dev's and the histogram equals the oracle's histogram of it,
    clamped into [lo, lo + n) for a wide and a narrow range; a ragged block row (19 blocks),
    values far outside the LDS bins (scale 0.013: the global-atomic path) and a table whose
    planes 1 and 2 differ (3 staged planes instead of plane 1 counted twice)."""
    torch = pytest.importorskip("torch")
    import ivclab_amd.device as D
    rng = np.random.default_rng(31 + 7 * zz + len(case))
    F, H, W, sr = 3, 48, 152, 4
    base = rng.integers(0, 256, (H + 16, W + 16)).astype(np.int16)
    frames = np.stack([np.clip(base[4 + f:4 + f + H, 2 * f:2 * f + W] + rng.integers(-9, 10, (H, W)),
                               0, 255) for f in range(F)]).astype(np.uint8)
    scale = {"jpeg": 1.0, "fine": 0.013, "custom": 0.5}[case]
    table = PatchQuant(scale).get_quantization_table().astype(np.float64)
    if case == "custom":
        table[2] *= 1.37
    fr = torch.from_numpy(frames).cuda()
    mv0 = torch.empty((F - 1, H // 8, W // 8), dtype=torch.int64, device="cuda")
    q0 = torch.empty((F - 1, H // 8, W // 8, 3, 64), dtype=torch.int32, device="cuda")
    D.inter_encode(fr, sr, table, mv0, q0, zigzag=bool(zz))
    for lo, n in [(-4097, 8194), (-3, 9)]:
        mv = torch.empty_like(mv0)
        q = torch.empty_like(q0)
        hist = torch.zeros(n, dtype=torch.int64, device="cuda")
        D.inter_encode(fr, sr, table, mv, q, zigzag=bool(zz), hist=hist, hist_lo=lo)
        torch.cuda.synchronize()
        assert_bits(q.cpu().numpy(), q0.cpu().numpy(), f"q {case} zz={zz}")
        assert_bits(mv.cpu().numpy(), mv0.cpu().numpy(), f"mv {case} zz={zz}")
        want = O.histogram(q0.cpu().numpy().reshape(-1), lo, n)
        assert np.array_equal(hist.cpu().numpy(), want), (case, zz, lo, n)
    if case == "fine":
        assert np.abs(q0.cpu().numpy()).max() > 600          # the out-of-range path ran
