"""Where a per-block call's time goes on this host: the C-ABI call through ctypes with prebuilt
arguments, the same call with nblk = 0 (argument checks only), and the drop-in class call."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ivclab_amd._native as N  # noqa: E402
from ivclab_amd import DiscreteCosineTransform, PatchQuant  # noqa: E402


def med(fn, reps=400, warm=50):
    for _ in range(warm):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return round(float(np.median(t)) * 1e6, 2)


L = N.lib()
rng = np.random.default_rng(1)
blk = rng.integers(0, 256, (8, 8)).astype(np.float64)
stk = rng.normal(0, 50, (3, 8, 8))
pq, dct = PatchQuant(1.0), DiscreteCosineTransform()
t = N.table_arg(pq.get_quantization_table())
qo = np.empty((1, 1, 3, 8, 8), np.int32)
do = np.empty((8, 8), np.float64)
pb, pt, pqo, pdo, ps = N.ptr(blk), N.ptr(t), N.ptr(qo), N.ptr(do), N.ptr(stk)
r = {
    "ctypes_noop_quantize_nblk0": med(lambda: L.ivc_quantize(ps, N.F64, 0, 3, pt, N.F64, pqo)),
    "ctypes_quantize": med(lambda: L.ivc_quantize(ps, N.F64, 1, 3, pt, N.F64, pqo)),
    "class_quantize": med(lambda: pq.quantize(stk)),
    "ctypes_dct": med(lambda: L.ivc_dct8x8(pb, N.F64, 1, pdo, N.F64, 0, 1)),
    "class_transform": med(lambda: dct.transform(blk)),
}
print(r)
