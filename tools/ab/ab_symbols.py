"""Same-process A/B timing of libivc variants (ab/*.so) on the symbol legs of bench.py: the
zero-run encode of the cfg3 zig-zag coefficients, the fused pixels -> symbols path (without and with the
emission pass's histogram), symbols -> RGB image, the symbol histogram and min/max.  Every variant's outputs are compared with the first one's.
    python tools/ab/ab_symbols.py ab/base.so ab/new.so [--frames 256] [--rounds 5]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ivclab_amd._native as N  # noqa: E402
import bench  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--frames", type=int, default=256)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--legs", default="", help="comma-separated subset of the legs")
ap.add_argument("--rccl", action="store_true",
                help="first create a one-rank RCCL process group (its streams take hardware queues, "
                     "as in bench.py --rccl)")
args = ap.parse_args()
if args.rccl:
    torch.cuda.set_device(0)
    from ivclab_amd.distributed import init_single_rank, global_histogram
    init_single_rank("cuda:0")
    _h = torch.zeros(8, dtype=torch.int64, device="cuda:0")
    global_histogram(_h, force=True)          # the communicator and its streams exist now
    torch.cuda.synchronize()
N.load_library()
libs = []
for p in args.libs:
    L = ctypes.CDLL(os.path.abspath(p))
    for name, (a, r) in N._SIGS.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = a, r
    libs.append((f"{len(libs)}:{os.path.basename(p)}", L))
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream().cuda_stream
t = N.table_arg(PatchQuant(1.0).get_quantization_table())
F, H, W = args.frames, 2160, 3840
img = bench.intra_frames(F, H, W, seed=3, dev=dev)
q = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
L0 = libs[0][1]
N.check(L0.ivc_intra_encode_dev(img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, N.F64, 1, q.data_ptr(),
                                None, 0, 0, stream))
nblk = q.numel() // 64
off = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
probe = torch.empty(1, dtype=torch.int32, device=dev)
N.check(L0.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(), probe.data_ptr(), 0, stream))
nsym = int(off[-1].item())
sym = torch.empty(nsym, dtype=torch.int32, device=dev)
# the stream (the decode leg's input, and the reference the encode legs must rewrite)
N.check(L0.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(), sym.data_ptr(), nsym, stream))
sym_ref = sym.clone()
nsd = torch.zeros(1, dtype=torch.int64, device=dev)
hist = torch.zeros(4200, dtype=torch.int64, device=dev)
mm = torch.empty(2, dtype=torch.int32, device=dev)
hist2 = torch.zeros(8194, dtype=torch.int64, device=dev)
rgb = torch.empty((F, H, W, 3), dtype=torch.float64, device=dev)
err = torch.zeros(3, dtype=torch.int64, device=dev)


def timeit(fn, reps=3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


legs = {
    "zerorun_encode": lambda L: N.check(L.ivc_zerorun_encode_dev(
        q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(), sym.data_ptr(), nsym, stream)),
    "intra_symbols": lambda L: N.check(L.ivc_intra_symbols_dev(
        img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, 4000, sym.data_ptr(), nsym, nsd.data_ptr(),
        stream)),
    "symbols_hist": lambda L: (hist2.zero_(), N.check(L.ivc_intra_symbols_hist_dev(
        img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, 4000, sym.data_ptr(), nsym, nsd.data_ptr(),
        hist2.data_ptr(), -4097, 8194, stream))),
    "symbols2image": lambda L: N.check(L.ivc_symbols2image_dev(
        sym.data_ptr(), nsym, F, H, W, 3, t.ctypes.data, 4000, 1, rgb.data_ptr(), err.data_ptr(),
        stream)),
    "histogram": lambda L: (hist.zero_(), N.check(L.ivc_histogram_i32_dev(
        sym.data_ptr(), nsym, -64, 4200, hist.data_ptr(), stream))),
    "minmax": lambda L: N.check(L.ivc_minmax_i32_dev(sym.data_ptr(), nsym, mm.data_ptr(), stream)),
}
if args.legs:
    legs = {k: v for k, v in legs.items() if k in args.legs.split(",")}
res = {(leg, n): [] for leg in legs for n, _ in libs}


def digest_of(x):
    """Whole-tensor checksum (chunked: int64 sum and an index-weighted sum of the words)."""
    v = x.view(-1)
    v = v.view(torch.int64) if v.dtype == torch.float64 else v
    s1 = s2 = 0
    CH = 1 << 26
    for i in range(0, v.numel(), CH):
        c = v[i:i + CH].to(torch.int64)
        w = (torch.arange(i, i + c.numel(), device=c.device, dtype=torch.int64) % 7919) + 1
        s1 += int(c.sum().item())
        s2 += int((c * w).sum().item())
    return (s1, s2, int(v.numel()))
check = {}
for rnd in range(args.rounds):
    for leg, fn in legs.items():
        for n, L in libs:
            res[(leg, n)].append(timeit(lambda: fn(L)))
            if rnd == 0:
                # outputs cleared, then one more call: a variant that leaves part of an output
                # unwritten cannot inherit the previous variant's values
                outs0 = {"zerorun_encode": sym, "intra_symbols": sym, "symbols_hist": hist2,
                         "symbols2image": rgb, "histogram": hist, "minmax": mm}
                if leg != "symbols2image":
                    outs0[leg].fill_(-3)
                else:
                    rgb.fill_(-3.0)
                fn(L)
                torch.cuda.synchronize()
                if leg in ("zerorun_encode", "intra_symbols", "symbols_hist") and not torch.equal(sym, sym_ref):
                    print(f"MISMATCH {leg} {n}: stream differs from the two-step stream", flush=True)
                if leg in ("zerorun_encode", "intra_symbols", "symbols_hist"):
                    sym.copy_(sym_ref)
                outs = {"zerorun_encode": sym, "intra_symbols": sym, "symbols_hist": hist2,
                        "symbols2image": rgb, "histogram": hist, "minmax": mm}
                digest = digest_of(outs[leg])
                check.setdefault(leg, digest)
                if digest != check[leg]:
                    print(f"MISMATCH {leg} {n}: {digest} vs {check[leg]}", flush=True)
for leg in legs:
    for n, _ in libs:
        v = res[(leg, n)]
        print(f"{leg:15s} {n:16s} median {float(np.median(v)):7.3f} ms  min {min(v):7.3f}", flush=True)
print(f"symbols {nsym}, blocks {nblk}")
