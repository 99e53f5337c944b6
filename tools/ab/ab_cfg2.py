"""Same-process A/B of libivc variants (ab/*.so, tools/ab/build_variant.py) on cfg2 (BASELINE
configs[1]: 1920x1080 RGB u8 -> per-channel DCT + quant + zig-zag, fused_encode_kernel C = 3):
one frame per launch and a 64-frame batch per launch, timed with HIP events in interleaved
rounds on the same device buffers; every variant's output is compared with the first one's.
    python tools/ab/ab_cfg2.py ab/base.so ab/new.so [--frames 64] [--rounds 5]"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ivclab_amd._native as N  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--pace", default="", help="comma-separated start rates (GB/s, 0 = off) per library")
args = ap.parse_args()

N.load_library()
libs = []
for p in args.libs:
    L = ctypes.CDLL(os.path.abspath(p))
    for name, (a, r) in N._SIGS.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = a, r
    for pc in [float(x) for x in args.pace.split(",") if x] or [None]:
        libs.append((f"{len(libs)}:{os.path.basename(p)}" + ("" if pc is None else f"@{pc:g}"), L, pc))

dev = torch.device("cuda:0")
t = N.table_arg(PatchQuant(1.0).get_quantization_table())
stream = torch.cuda.current_stream().cuda_stream
F, H, W = args.frames, 1080, 1920
g = torch.Generator(device=dev)
g.manual_seed(1)
frames = torch.randint(0, 256, (F, H, W, 3), device=dev, generator=g, dtype=torch.uint8)
out = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)


def call(L, nf):
    st = L.ivc_intra_encode_dev(frames.data_ptr(), 1, nf, H, W, 3, N.ptr(t), 10, 1, out.data_ptr(),
                                None, 0, 0, stream)
    assert st == 0, st


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


res = {n: {"one": [], "batch": []} for n, _, _ in libs}
ref = None
for rnd in range(args.rounds):
    for name, L, pc in libs:
        if pc is not None and hasattr(L, "ivc_set_store_pace"):
            L.ivc_set_store_pace(ctypes.c_double(pc))
        res[name]["one"].append(timeit(lambda: call(L, 1), 200))
        res[name]["batch"].append(timeit(lambda: call(L, F), 20))
        if rnd == 0:
            out.fill_(-7)
            call(L, F)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            else:
                print(name, "identical" if torch.equal(out, ref) else "DIFFERS")
algo_one, algo_b = H * W * 15, F * H * W * 15
for name, r in res.items():
    one, b = min(r["one"]), min(r["batch"])
    print(f"{name:32s} one_frame {one * 1e3:7.2f} us ({algo_one / one / 1e6 / 8000:.3f})  "
          f"batch_{F} {b:.4f} ms ({algo_b / b / 1e6 / 8000:.3f})  all one {[round(x * 1e3, 1) for x in r['one']]} "
          f"batch {[round(x, 4) for x in r['batch']]}")
