"""Same-process A/B timing of libivc variants (ab/*.so) on the exact-u8 +-16 motion search
alone (ivc_motion_estimate_dev, IVC_ME_EXACT_U8: the matrix-core search me_mfma16_kernel)
over the cfg4 sequence (1080p x 300, 299 pairs) and one 8K chunk (9 frames); interleaved
rounds, HIP events on the current stream; every variant's vectors are compared with the first
variant's bit for bit (and, with --oracle, pair 0 with the C oracle).
    python tools/ab/ab_me.py ab/base.so ab/new.so [--rounds 5]"""
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

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--oracle", action="store_true")
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
cases = {"1080p_x300": bench.inter_frames(300, 1080, 1920, seed=4, dev=dev),
         "8k_x9": bench.inter_frames(9, 4320, 7680, seed=5, dev=dev)}
res, ref = {}, {}
for rnd in range(args.rounds):
    for cname, seq in cases.items():
        F, H, W = seq.shape
        mv = torch.empty((F - 1, H // 8, W // 8), dtype=torch.int64, device=dev)
        for n, L in libs:
            call = lambda: N.check(L.ivc_motion_estimate_dev(seq.data_ptr(), seq[1:].data_ptr(),
                                                             N.DTYPE_CODE[np.dtype(np.uint8)], F - 1,
                                                             H, W, 16, N.ME_EXACT_U8,
                                                             mv.data_ptr(), stream))
            mv.fill_(-1)
            call()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                call()
            e.record()
            torch.cuda.synchronize()
            res.setdefault((cname, n), []).append(s.elapsed_time(e) / args.reps)
            if rnd == 0:
                host = mv.cpu()
                if cname not in ref:
                    ref[cname] = host
                    if args.oracle and H <= 1080:
                        from oracle import c_motion_vectors
                        want = c_motion_vectors(seq[0].cpu().numpy(), seq[1].cpu().numpy(), 16,
                                                exact_u8=True)
                        ok = np.array_equal(host[0].numpy(), want.reshape(host[0].shape))
                        print(f"oracle pair 0 {cname}: {'ok' if ok else 'MISMATCH'}", flush=True)
                elif not torch.equal(host, ref[cname]):
                    bad = int((host != ref[cname]).sum())
                    print(f"MISMATCH {cname} {n}: {bad} vectors differ", flush=True)
        del mv
for (cname, n), v in res.items():
    print(f"{cname:11s} {n:14s} median {float(np.median(v)):8.3f} ms  min {min(v):8.3f}", flush=True)
