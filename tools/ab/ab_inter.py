"""Same-process A/B timing of libivc variants (ab/*.so) on the fused inter encoder
(ivc_inter_encode_dev: ME + MC + residual DCT/quant) over one cfg5 chunk (9 frames of the
bench's 8K sequence = 8 pairs) and the cfg4 1080p x 300 sequence; interleaved rounds, HIP
events; every variant's mv and q are compared with the first one's.
    python tools/ab/ab_inter.py ab/base.so ab/new.so [--rounds 5]"""
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
ap.add_argument("--rounds", type=int, default=5)
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
t = N.table_arg(PatchQuant(1.0).get_quantization_table())
cases = {"8k_x9": bench.inter_frames(9, 4320, 7680, seed=5, dev=dev),
         "1080p_x300": bench.inter_frames(300, 1080, 1920, seed=4, dev=dev)}
res = {}
ref = {}
for rnd in range(args.rounds):
    for cname, seq in cases.items():
        F, H, W = seq.shape
        for n, L in libs:
            mv = torch.empty((F - 1, H // 8, W // 8), dtype=torch.int64, device=dev)
            q = torch.empty((F - 1, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
            call = lambda: N.check(L.ivc_inter_encode_dev(seq.data_ptr(), F, H, W, 16, t.ctypes.data,
                                                          N.F64, 0, mv.data_ptr(), q.data_ptr(), stream))
            call()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                call()
            e.record()
            torch.cuda.synchronize()
            res.setdefault((cname, n), []).append(s.elapsed_time(e) / 3)
            if rnd == 0:
                dg = (int(mv.sum().item()), int(q.to(torch.int64).sum().item()))
                ref.setdefault(cname, dg)
                if dg != ref[cname]:
                    print(f"MISMATCH {cname} {n}: {dg} vs {ref[cname]}", flush=True)
            del mv, q
for (cname, n), v in res.items():
    print(f"{cname:11s} {n:14s} median {float(np.median(v)):8.3f} ms  min {min(v):8.3f}", flush=True)
