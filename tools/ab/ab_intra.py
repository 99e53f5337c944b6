"""Same-process A/B timing of libivc variants (ab/*.so, tools/ab/build_variant.sh) on the
bench workloads: each variant's ivc_intra_encode_dev (cfg3) and ivc_inter_encode_dev (cfg4)
are timed with HIP events in interleaved rounds on the same device buffers, and every
variant's output is compared with the first one's.
    python tools/ab/ab_intra.py ab/base.so ab/new.so [--frames 256] [--rounds 5] [--inter]"""
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
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--inter", action="store_true")
args = ap.parse_args()

N.load_library()                      # binds torch's HIP runtime first
libs = []
for p in args.libs:
    L = ctypes.CDLL(os.path.abspath(p))
    for name, (a, r) in N._SIGS.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = a, r
    libs.append((f"{len(libs)}:{os.path.basename(p)}", L))

dev = torch.device("cuda:0")
t = N.table_arg(PatchQuant(1.0).get_quantization_table())
stream = torch.cuda.current_stream().cuda_stream


def timeit(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(args.reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / args.reps


F, H, W = args.frames, 2160, 3840
img = bench.intra_frames(F, H, W, seed=3, dev=dev)
outs = [torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev) for _ in libs]
res = {n: [] for n, _ in libs}
for _ in range(args.rounds):
    for (n, L), o in zip(libs, outs):
        res[n].append(timeit(lambda: N.check(L.ivc_intra_encode_dev(
            img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, N.F64, 0, o.data_ptr(), None, 0, 0,
            stream))))
for (n, _), o in zip(libs, outs):
    same = bool(torch.equal(o, outs[0]))
    med = float(np.median(res[n]))
    print(f"intra {n:24s} median {med:7.3f} ms  min {min(res[n]):7.3f}  "
          f"{F * H * W * 13 / med / 1e6:7.1f} GB/s  same_as_first={same}", flush=True)
del outs, img
torch.cuda.empty_cache()

if args.inter:
    Fi, Hi, Wi, sr = 300, 1080, 1920, 16
    seq = bench.inter_frames(Fi, Hi, Wi, seed=4, dev=dev)
    mvs = [torch.empty((Fi - 1, Hi // 8, Wi // 8), dtype=torch.int64, device=dev) for _ in libs]
    qs = [torch.empty((Fi - 1, Hi // 8, Wi // 8, 3, 64), dtype=torch.int32, device=dev) for _ in libs]
    res = {n: [] for n, _ in libs}
    for _ in range(args.rounds):
        for (n, L), mv, q in zip(libs, mvs, qs):
            res[n].append(timeit(lambda: N.check(L.ivc_inter_encode_dev(
                seq.data_ptr(), Fi, Hi, Wi, sr, t.ctypes.data, N.F64, 0, mv.data_ptr(),
                q.data_ptr(), stream))))
    for (n, _), mv, q in zip(libs, mvs, qs):
        same = bool(torch.equal(mv, mvs[0]) and torch.equal(q, qs[0]))
        med = float(np.median(res[n]))
        print(f"inter {n:24s} median {med:7.3f} ms  min {min(res[n]):7.3f}  same_as_first={same}",
              flush=True)
