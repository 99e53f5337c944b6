"""Vector-by-vector comparison of libivc variants' exact-u8 +-16 search on the bench's cfg5
sequence (8K x 120, 119 pairs in one call) and a repeat of each (determinism); then the
unchunked inter_encode histogram of each library (its sha256 against the round-4 value).
    python tools/ab/ab_me_seq.py ab/a.so ab/b.so ..."""
import ctypes
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ivclab_amd._native as N  # noqa: E402
import bench  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402

N.load_library()
libs = []
for p in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(p))
    for name, (a, r) in N._SIGS.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = a, r
    libs.append((os.path.basename(p), L))
dev = torch.device("cuda:0")
s = torch.cuda.current_stream().cuda_stream
F, H, W, sr = int(os.environ.get("SEQ_FRAMES", "120")), 4320, 7680, 16
seq = bench.inter_frames(F, H, W, seed=5, dev=dev)
ref = None
for name, L in libs:
    outs = []
    for rep in range(2):
        mv = torch.full((F - 1, H // 8, W // 8), -1, dtype=torch.int64, device=dev)
        N.check(L.ivc_motion_estimate_dev(seq.data_ptr(), seq[1:].data_ptr(), 1, F - 1, H, W, sr,
                                          N.ME_EXACT_U8, mv.data_ptr(), s))
        torch.cuda.synchronize()
        outs.append(mv)
    det = torch.equal(outs[0], outs[1])
    msg = f"{name}: repeat {'identical' if det else 'DIFFERS (%d)' % int((outs[0] != outs[1]).sum())}"
    if ref is None:
        ref = outs[0]
    else:
        d = outs[0] != ref
        nd = int(d.sum())
        msg += f"; vs first lib: {'identical' if nd == 0 else 'DIFFERS in %d vectors' % nd}"
        if nd:
            idx = torch.nonzero(d)[:8].tolist()
            msg += f" first {idx}"
    print(msg, flush=True)
    del outs
table = N.table_arg(PatchQuant(1.0).get_quantization_table())
nmv = (2 * sr + 1) ** 2
for name, L in libs:
    mvf = torch.empty((F - 1, H // 8, W // 8), dtype=torch.int64, device=dev)
    qf = torch.empty((F - 1, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    hs = []
    for rep in range(2):
        hf = torch.zeros(bench.HIST_BINS + nmv, dtype=torch.int64, device=dev)
        N.check(L.ivc_inter_encode_dev(seq.data_ptr(), F, H, W, sr, N.ptr(table), 10, 0, mvf.data_ptr(),
                                       qf.data_ptr(), s))
        N.check(L.ivc_histogram_i32_dev(qf.data_ptr(), qf.numel(), bench.HIST_LO, bench.HIST_BINS,
                                    hf.data_ptr(), s))
        N.check(L.ivc_histogram_i64_dev(mvf.data_ptr(), mvf.numel(), 0, nmv,
                                        hf[bench.HIST_BINS:].data_ptr(), s))
        torch.cuda.synchronize()
        hs.append(hashlib.sha256(hf.cpu().numpy().tobytes()).hexdigest()[:16])
    print(f"{name}: unchunked inter_encode histogram sha {hs} (r04: 4b7728afae1f916c)", flush=True)
    del mvf, qf
