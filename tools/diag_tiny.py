"""Step-by-step probe of the tiny host-call path (prints each step before it runs)."""
import faulthandler
import sys

import numpy as np

faulthandler.enable()


def step(msg):
    print(msg, flush=True)


step("import")
sys.path.insert(0, ".")
import ivclab_amd._native as N  # noqa: E402

step("load")
L = N.lib()
blk = (np.arange(64) * 7 % 256).astype(np.uint8).reshape(8, 8)
out = np.empty((8, 8), np.float64)
step("dct8x8 u8 tiny")
N.check(L.ivc_dct8x8(N.ptr(blk), 1, 1, N.ptr(out), N.F64, 0, N.NORM_CODE["ortho"]), "dct")
step(f"ok {out[0, :3]}")
q = np.linspace(-300, 300, 192).reshape(3, 8, 8)
t = np.full(192, 17.0)
qo = np.empty((3, 8, 8), np.int32)
step("quantize f64 tiny")
N.check(L.ivc_quantize(N.ptr(q), N.F64, 1, 3, N.ptr(t), N.F64, N.ptr(qo)), "quantize")
step(f"ok {qo.ravel()[:4]}")
