"""Same-process A/B of libivc variants on the zero-run encoder (ivc_zerorun_encode_dev) over
the cfg3 zig-zag output (256 x 4K luma -> [F,h,w,3,64] int32): interleaved rounds on one
input buffer, HIP events on the current stream; every variant's symbols and block offsets
are compared with the first variant's.
    python tools/ab/ab_zr.py ab/base.so ab/new.so [--frames 256] [--rounds 5]"""
import argparse
import ctypes
import os
import sys

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
args = ap.parse_args()

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
F, H, W = args.frames, 2160, 3840
frames = bench.intra_frames(F, H, W, seed=3, dev=dev)
q = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
t = N.table_arg(PatchQuant(1.0).get_quantization_table())
L0 = libs[0][1]
N.check(L0.ivc_intra_encode_dev(frames.data_ptr(), 1, F, H, W, 1, t.ctypes.data, N.F64, 1,
                                q.data_ptr(), None, 0, 0, stream), "intra_encode_dev")
nblk = q.numel() // 64
off = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
cap = nblk * 98
# size the stream once
out = torch.empty(1, dtype=torch.int32, device=dev)
N.check(L0.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(), out.data_ptr(),
                                  0, stream), "zerorun")
torch.cuda.synchronize()
total = int(off[-1].item())
out = torch.empty(total, dtype=torch.int32, device=dev)
ref_out = ref_off = None
print(f"blocks {nblk}, symbols {total}", flush=True)


def run(L):
    N.check(L.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(), out.data_ptr(),
                                     total, stream), "zerorun")


times = {name: [] for name, _ in libs}
for rd in range(args.rounds):
    for name, L in libs:
        off.fill_(-1)
        out.fill_(-7)
        run(L)
        torch.cuda.synchronize()
        if ref_out is None:
            ref_out, ref_off = out.clone(), off.clone()
        else:
            ok = torch.equal(out, ref_out) and torch.equal(off, ref_off)
            if not ok:
                print(f"MISMATCH {name}", flush=True)
                sys.exit(3)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.reps):
            run(L)
        e.record()
        torch.cuda.synchronize()
        times[name].append(s.elapsed_time(e) / args.reps)
    print(f"round {rd}: " + "  ".join(f"{n} {times[n][-1]:.3f}" for n, _ in libs), flush=True)
for name, _ in libs:
    ts = sorted(times[name])
    print(f"zerorun {name}: median {ts[len(ts) // 2]:.3f} ms  min {ts[0]:.3f}", flush=True)
