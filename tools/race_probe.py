"""Repeat bench.py's cfg5 sharded step (ME + residual encode with the fused coefficient
histogram, 8-pair chunks, the MV histograms on a side stream) and compare every run's mv, q
and histogram bitwise with the first run's and with one unchunked, single-stream run; on a
mismatch print where (pair, block row, block column) and in which tensor.  Diagnostic for an
intermittent histogram mismatch (profiles/r05_race.md).

  python tools/race_probe.py [--reps 12] [--frames 120] [--mode chunked|unchunked|noside|intra]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402
import ivclab_amd.device as D  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402
from ivclab_amd import _native as N  # noqa: E402


def where(a, b, name):
    ne = (a != b)
    if a.dim() > 3:
        ne = ne.flatten(3).any(-1)
    idx = ne.nonzero()
    print(f"  {name}: {idx.shape[0]} mismatching (pair, by, bx) entries; first {idx[:8].tolist()}",
          flush=True)
    pairs = idx[:, 0].unique().tolist()
    print(f"  {name}: pairs {pairs[:20]}", flush=True)


def ssd_report(seq, mv, mvr, sr, limit=6):
    """the wrong and the right candidate of each mismatching block with both SSDs"""
    N_ = 2 * sr + 1
    idx = (mv != mvr).nonzero()[:limit].tolist()
    for p, by, bx in idx:
        ref = seq[p].to(torch.int64)
        cur = seq[p + 1].to(torch.int64)
        blk = cur[8 * by:8 * by + 8, 8 * bx:8 * bx + 8]
        out = []
        for v in (int(mv[p, by, bx]), int(mvr[p, by, bx])):
            dy, dx = v // N_ - sr, v % N_ - sr
            y, x = 8 * by + dy, 8 * bx + dx
            ok = 0 <= y <= ref.shape[0] - 8 and 0 <= x <= ref.shape[1] - 8
            s = int(((ref[y:y + 8, x:x + 8] - blk) ** 2).sum()) if ok else None
            out.append((v, dy, dx, s))
        print(f"  block ({p}, {by}, {bx}): got {out[0]}  want {out[1]}", flush=True)


def intra(args, dev):
    """cfg3 (256 x 4K luma): the pipelined pixels -> symbols call with its histogram, the
    pipelined zero-run encode and the pipelined symbols -> image call, each run compared bit
    for bit with the two-step stream / the first run's outputs"""
    L = N.lib()
    stream = torch.cuda.current_stream().cuda_stream
    t = N.table_arg(PatchQuant(1.0).get_quantization_table())
    F, H, W = 256, 2160, 3840
    img = B.intra_frames(F, H, W, seed=3, dev=dev)
    q = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    N.check(L.ivc_intra_encode_dev(img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, N.F64, 1,
                                   q.data_ptr(), None, 0, 0, stream))
    nblk = q.numel() // 64
    off = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
    one = torch.empty(1, dtype=torch.int32, device=dev)
    N.check(L.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(),
                                     one.data_ptr(), 0, stream))
    nsym = int(off[-1].item())
    ref = torch.empty(nsym, dtype=torch.int32, device=dev)
    N.check(L.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(),
                                     ref.data_ptr(), nsym, stream))
    work = torch.empty_like(ref)
    nsd = torch.zeros(1, dtype=torch.int64, device=dev)
    hist = torch.zeros(8194, dtype=torch.int64, device=dev)
    rgb = torch.empty((F, H, W, 3), dtype=torch.float64, device=dev)
    err = torch.zeros(3, dtype=torch.int64, device=dev)
    hist_ref = rgb_ref = None
    bad = 0
    for rep in range(args.reps):
        hist.zero_()
        N.check(L.ivc_intra_symbols_hist_dev(img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, 4000,
                                             work.data_ptr(), nsym, nsd.data_ptr(),
                                             hist.data_ptr(), -4097, 8194, stream))
        ok_s = torch.equal(work, ref) and int(nsd.item()) == nsym
        N.check(L.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(),
                                         work.data_ptr(), nsym, stream))
        ok_z = torch.equal(work, ref)
        N.check(L.ivc_symbols2image_dev(ref.data_ptr(), nsym, F, H, W, 3, t.ctypes.data, 4000, 1,
                                        rgb.data_ptr(), err.data_ptr(), stream))
        torch.cuda.synchronize()
        if rep == 0:
            hist_ref, rgb_ref = hist.clone(), rgb.clone()
        ok_h = torch.equal(hist, hist_ref)
        ok_d = torch.equal(rgb.view(torch.int64), rgb_ref.view(torch.int64)) and int(err[0]) == 0
        ok = ok_s and ok_z and ok_h and ok_d
        if not args.quiet or not ok:
            print(f"rep {rep}: image2symbols {'ok' if ok_s else 'DIFF'}  zerorun {'ok' if ok_z else 'DIFF'}  "
                  f"hist {'ok' if ok_h else 'DIFF'}  symbols2image {'ok' if ok_d else 'DIFF'}", flush=True)
        if not ok_d:
            ne = (rgb.view(torch.int64) != rgb_ref.view(torch.int64)).any(-1).nonzero()
            print(f"  symbols2image: {ne.shape[0]} pixels differ, first {ne[:6].tolist()}", flush=True)
        bad += not ok
    print(f"mode intra lib {args.lib or 'in-tree'}: {bad} of {args.reps} runs differ", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--mode", default="chunked")
    ap.add_argument("--lib", default=None, help="a libivc variant (ab/*.so) instead of the in-tree one")
    ap.add_argument("--quiet", action="store_true", help="print only the runs that differ")
    args = ap.parse_args()
    if args.lib:
        import ctypes
        N.load_library()
        L = ctypes.CDLL(os.path.abspath(args.lib))
        for name, (a, r) in N._SIGS.items():
            fn = getattr(L, name, None)
            if fn is not None:
                fn.argtypes, fn.restype = a, r
        N._lib = L
    dev = torch.device("cuda", 0)
    if args.mode == "intra":
        return intra(args, dev)
    F, H, W, sr = args.frames, 4320, 7680, 16
    table = PatchQuant(1.0).get_quantization_table()
    seq = B.inter_frames(F, H, W, seed=5, dev=dev)
    P = F - 1
    nmv = (2 * sr + 1) ** 2
    mv = torch.empty((P, H // 8, W // 8), dtype=torch.int64, device=dev)
    q = torch.empty((P, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    hist = torch.zeros(B.HIST_BINS + nmv, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(device=dev)
    # the independent reference: one unchunked call on the main stream, main-stream histograms
    mvr = torch.empty_like(mv)
    qr = torch.empty_like(q)
    D.inter_encode(seq, sr, table, mvr, qr)
    hr = torch.zeros_like(hist)
    D.histogram(qr.view(-1), B.HIST_LO, hr[:B.HIST_BINS])
    D.histogram(mvr.view(-1), 0, hr[B.HIST_BINS:])
    torch.cuda.synchronize()
    if args.mode == "chunked":
        step = B.make_sharded_step(D, N, seq, P, sr, table, mv, q, hist, 8, 2, False, side)
    elif args.mode == "noside":
        step = B.make_sharded_step(D, N, seq, P, sr, table, mv, q, hist, 8, 2, False,
                                   torch.cuda.current_stream())
    else:
        def step():
            hist.zero_()
            D.inter_encode(seq, sr, table, mv, q, hist=hist[:B.HIST_BINS], hist_lo=B.HIST_LO)
            D.histogram(mv.view(-1), 0, hist[B.HIST_BINS:])
            return hist
    bad = 0
    for rep in range(args.reps):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        okm, okq, okh = torch.equal(mv, mvr), torch.equal(q, qr), torch.equal(hist, hr)
        if not args.quiet or not (okm and okq and okh):
            print(f"rep {rep}: {ms:.1f} ms  mv {'ok' if okm else 'DIFF'}  q {'ok' if okq else 'DIFF'}  "
                  f"hist {'ok' if okh else 'DIFF'}", flush=True)
        if not okm:
            where(mv, mvr, "mv")
            ssd_report(seq, mv, mvr, sr)
        if not okq:
            where(q, qr, "q")
        if not okh:
            d = (hist - hr).nonzero().flatten()
            print(f"  hist: {d.numel()} bins differ, first {d[:10].tolist()} "
                  f"(coef bins < {B.HIST_BINS}), deltas {(hist - hr)[d[:10]].tolist()}", flush=True)
        bad += not (okm and okq and okh)
    print(f"mode {args.mode} lib {args.lib or 'in-tree'}: {bad} of {args.reps} runs differ", flush=True)


if __name__ == "__main__":
    main()
