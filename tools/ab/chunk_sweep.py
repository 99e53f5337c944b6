"""Chunk-count sweep of the pipelined calls through the tuning API (ivc_set_tuning), one
process, interleaved rounds, HIP events; every count's output is compared with the first
count's (digest of the whole output) — the chunking must not change a bit.
    python tools/ab/chunk_sweep.py --leg symbols2image --counts 16,24,32,48,64 [--rounds 5]
        [--lags 1,2,3]  (symbols2image: IVC_TUNE_S2I_LAG values crossed with the counts)
        [--lib ab/variant.so]  (a built variant instead of the in-tree library)
Legs: symbols2image (IVC_TUNE_S2I_CHUNKS), zerorun (IVC_TUNE_ZR_CHUNKS), symbols_hist
(IVC_TUNE_SYM_CHUNKS) on the cfg3 batch (256 x 4K luma)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import ivclab_amd._native as N  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402

KEYS = {"zerorun": 0, "symbols_hist": 1, "symbols2image": 2}

ap = argparse.ArgumentParser()
ap.add_argument("--leg", default="symbols2image", choices=sorted(KEYS))
ap.add_argument("--counts", default="16,24,32,48,64")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--lags", default="0")
ap.add_argument("--lib", default=None)
args = ap.parse_args()
counts = [(int(c), int(g)) for c in args.counts.split(",") for g in args.lags.split(",")]
LAG_KEY = 7
if args.lib:
    N.load_library(os.path.abspath(args.lib))
    assert N.load_library()._name == os.path.abspath(args.lib), "the in-tree library was loaded first"
L = N.lib()
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream().cuda_stream
t = N.table_arg(PatchQuant(1.0).get_quantization_table())
F, H, W = 256, 2160, 3840
img = bench.intra_frames(F, H, W, seed=3, dev=dev)
q = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
N.check(L.ivc_intra_encode_dev(img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, N.F64, 1, q.data_ptr(),
                               None, 0, 0, stream))
nblk = q.numel() // 64
off = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
one = torch.empty(1, dtype=torch.int32, device=dev)
N.check(L.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(), one.data_ptr(), 0, stream))
nsym = int(off[-1].item())
sym = torch.empty(nsym, dtype=torch.int32, device=dev)
N.check(L.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(), sym.data_ptr(), nsym, stream))
work = torch.empty_like(sym)
nsd = torch.zeros(1, dtype=torch.int64, device=dev)
hist = torch.zeros(8194, dtype=torch.int64, device=dev)
rgb = torch.empty((F, H, W, 3), dtype=torch.float64, device=dev)
err = torch.zeros(3, dtype=torch.int64, device=dev)
legs = {
    "zerorun": (lambda: N.check(L.ivc_zerorun_encode_dev(q.data_ptr(), nblk, 64, 64, 4000, off.data_ptr(),
                                                         work.data_ptr(), nsym, stream)), work),
    "symbols_hist": (lambda: (hist.zero_(), N.check(L.ivc_intra_symbols_hist_dev(
        img.data_ptr(), 1, F, H, W, 1, t.ctypes.data, 4000, work.data_ptr(), nsym, nsd.data_ptr(),
        hist.data_ptr(), -4097, 8194, stream))), work),
    "symbols2image": (lambda: N.check(L.ivc_symbols2image_dev(sym.data_ptr(), nsym, F, H, W, 3, t.ctypes.data,
                                                              4000, 1, rgb.data_ptr(), err.data_ptr(), stream)), rgb),
}
fn, out = legs[args.leg]


def digest(x):
    v = x.view(-1)
    v = v.view(torch.int64) if v.dtype == torch.float64 else v
    s1 = s2 = 0
    CH = 1 << 26
    for i in range(0, v.numel(), CH):
        c = v[i:i + CH].to(torch.int64)
        w = (torch.arange(i, i + c.numel(), device=c.device, dtype=torch.int64) % 7919) + 1
        s1 += int(c.sum().item())
        s2 += int((c * w).sum().item())
    return s1, s2


key = KEYS[args.leg]
prev = L.ivc_tuning(key)
use_lag = args.lags != "0"      # (the IVC_TUNE_S2I_LAG key exists only in r06ab's builds)
prev_lag = L.ivc_tuning(LAG_KEY) if use_lag else 0
res = {c: [] for c in counts}
ref = None
try:
    for rnd in range(args.rounds):
        for c in counts:
            N.check(L.ivc_set_tuning(key, c[0]))
            if use_lag:
                N.check(L.ivc_set_tuning(LAG_KEY, c[1]))
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[c].append(s.elapsed_time(e) / 3)
            if rnd == 0:
                d = digest(out)
                ref = ref or d
                if d != ref:
                    print(f"MISMATCH {args.leg} chunks={c[0]} lag={c[1]}", flush=True)
finally:
    N.check(L.ivc_set_tuning(key, prev))
    if use_lag:
        N.check(L.ivc_set_tuning(LAG_KEY, prev_lag))
for c in counts:
    v = sorted(res[c])
    print(f"{args.leg:14s} {args.lib or 'in-tree'} chunks {c[0]:3d} lag {c[1]:2d}  median {v[len(v) // 2]:7.3f} ms  "
          f"min {v[0]:7.3f}", flush=True)
