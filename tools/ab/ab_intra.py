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
ap.add_argument("--inter-shape", default="300x1080x1920", help="frames x H x W of the inter A/B")
ap.add_argument("--pace", default="", help="comma-separated store-pace rates (GB/s, 0 = off) "
                "to time for every library that exports ivc_set_store_pace")
ap.add_argument("--trace-pace", type=int, default=0,
                help="then trace N consecutive adaptive launches per paced library")
ap.add_argument("--trace-start", default="6000", help="starting rates of the traces")
args = ap.parse_args()

N.load_library()                      # binds torch's HIP runtime first
libs = []
for p in args.libs:
    L = ctypes.CDLL(os.path.abspath(p))
    for name, (a, r) in N._SIGS.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = a, r
    paces = [float(x) for x in args.pace.split(",") if x] if hasattr(L, "ivc_set_store_pace") else []
    for pc in paces or [None]:
        tag = "" if pc is None else f"@{pc:g}"
        libs.append((f"{len(libs)}:{os.path.basename(p)}{tag}", (L, pc)))

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


def timeit_once(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


F, H, W = args.frames, 2160, 3840
img = bench.intra_frames(F, H, W, seed=3, dev=dev)
# one output buffer for every variant (separate buffers showed placement-dependent timings);
# the first variant's output is kept as the reference
o = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
ref, same = None, {}
res = {n: [] for n, _ in libs}
fill = []
for rnd in range(args.rounds):
    fill.append(timeit(lambda: o.fill_(0)))
    for n, (L, pc) in libs:
        if pc is not None:
            N.check(L.ivc_set_store_pace(pc))
        res[n].append(timeit(lambda: N.check(L.ivc_intra_encode_dev(
            img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, N.F64, 0, o.data_ptr(), None, 0, 0,
            stream))))
        if rnd == 0:
            if ref is None:
                ref = o.clone()
            same[n] = bool(torch.equal(o, ref))
for n, _ in libs:
    med = float(np.median(res[n]))
    print(f"intra {n:24s} median {med:7.3f} ms  min {min(res[n]):7.3f}  "
          f"{F * H * W * 13 / med / 1e6:7.1f} GB/s  same_as_first={same[n]}", flush=True)
print(f"torch fill_ of the same output buffer: median {float(np.median(fill)):7.3f} ms "
      f"({o.numel() * 4 / float(np.median(fill)) / 1e6:7.1f} GB/s)", flush=True)
if args.trace_pace:
    # adaptive pacing: consecutive launches from each starting rate, one line per launch
    seen = set()
    for n, (L, pc) in libs:
        if not hasattr(L, "ivc_store_pace_late") or id(L) in seen:
            continue
        seen.add(id(L))
        for start in [float(x) for x in args.trace_start.split(",")]:
            N.check(L.ivc_set_store_pace(start))
            line = []
            for i in range(args.trace_pace):
                ms = timeit_once(lambda: N.check(L.ivc_intra_encode_dev(
                    img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, N.F64, 0, o.data_ptr(), None, 0,
                    0, stream)))
                line.append(f"{ms:.3f}@{L.ivc_store_pace():.0f}/{L.ivc_store_pace_late():.3f}")
            print(f"trace {n} start {start:g}: " + " ".join(line), flush=True)
del o, ref
del img
torch.cuda.empty_cache()

if args.inter:
    Fi, Hi, Wi = map(int, args.inter_shape.split("x"))
    sr = 16
    seq = bench.inter_frames(Fi, Hi, Wi, seed=4, dev=dev)
    mvs = [torch.empty((Fi - 1, Hi // 8, Wi // 8), dtype=torch.int64, device=dev) for _ in libs]
    qs = [torch.empty((Fi - 1, Hi // 8, Wi // 8, 3, 64), dtype=torch.int32, device=dev) for _ in libs]
    res = {n: [] for n, _ in libs}
    for _ in range(args.rounds):
        for (n, (L, pc)), mv, q in zip(libs, mvs, qs):
            if pc is not None:
                N.check(L.ivc_set_store_pace(pc))
            res[n].append(timeit(lambda: N.check(L.ivc_inter_encode_dev(
                seq.data_ptr(), Fi, Hi, Wi, sr, t.ctypes.data, N.F64, 0, mv.data_ptr(),
                q.data_ptr(), stream))))
    for (n, _), mv, q in zip(libs, mvs, qs):
        same = bool(torch.equal(mv, mvs[0]) and torch.equal(q, qs[0]))
        med = float(np.median(res[n]))
        print(f"inter {n:24s} median {med:7.3f} ms  min {min(res[n]):7.3f}  same_as_first={same}",
              flush=True)
