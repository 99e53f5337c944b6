"""CPU oracle for the ivclab block-codec hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / the timed CPU baseline.  The product (ivclab_amd/) never
imports it and has no CPU fallback.

Contents
  ivc_oracle.py   NumPy/SciPy restatement of the reference methods on the hot path, each
                  function citing the reference file:line it follows.  Pinned against the
                  golden vectors in tests/golden/ (generated from the reference itself by
                  tests/golden/make_golden.py), see tests/test_oracle_golden.py.
  ivc_oracle.c    plain-C restatement of motion estimation / compensation (NumPy SSD
                  order), for parity checks at sizes where the Python loop is too slow.
                  Built by oracle/Makefile into oracle/_build/libivc_oracle.so.
"""

import ctypes as _ct
import os as _os
import subprocess as _sp

_HERE = _os.path.dirname(_os.path.abspath(__file__))
_clib = None


def clib():
    """Load (building on first use with gcc if needed) oracle/_build/libivc_oracle.so."""
    global _clib
    if _clib is None:
        so = _os.path.join(_HERE, "_build", "libivc_oracle.so")
        src = _os.path.join(_HERE, "ivc_oracle.c")
        if not _os.path.exists(so) or _os.path.getmtime(so) < _os.path.getmtime(src):
            _sp.run(["make", "-s", "-C", _HERE], check=True)
        lib = _ct.CDLL(so)
        P, L, I = _ct.c_void_p, _ct.c_long, _ct.c_int
        lib.oracle_me.argtypes = [P, P, I, I, L, L, I, L, L, P]
        lib.oracle_me.restype = I
        lib.oracle_mc.argtypes = [P, I, L, L, L, P, I, P]
        lib.oracle_mc.restype = None
        _clib = lib
    return _clib


_DT = {"uint8": 1, "int8": 2, "uint16": 3, "int16": 4, "uint32": 5, "int32": 6,
       "uint64": 7, "int64": 8, "float32": 9, "float64": 10}


def c_motion_vectors(ref, cur, sr, exact_u8=False, rows=None):
    """C restatement of motion.py:8-58 for one frame pair; rows=(by0, by1) restricts the
    block rows computed (candidate validity still uses the full frame)."""
    import numpy as np
    ref = np.ascontiguousarray(ref)
    cur = np.ascontiguousarray(cur, dtype=ref.dtype)
    H, W = ref.shape
    by0, by1 = rows if rows is not None else (0, H // 8)
    mv = np.zeros((by1 - by0, W // 8), dtype=np.int64)
    rc = clib().oracle_me(ref.ctypes.data, cur.ctypes.data, _DT[ref.dtype.name],
                          1 if exact_u8 else 0, H, W, sr, by0, by1, mv.ctypes.data)
    if rc != 0:
        raise TypeError(f"oracle_me: unsupported dtype {ref.dtype}")
    return mv[..., None]


def c_motion_compensate(ref, mv, sr):
    """C restatement of motion.py:60-97 for one [H,W,C] frame."""
    import numpy as np
    ref = np.ascontiguousarray(ref)
    H, W, C = ref.shape
    out = np.empty_like(ref)
    mvc = np.ascontiguousarray(mv, dtype=np.int64)
    clib().oracle_mc(ref.ctypes.data, ref.itemsize, H, W, C, mvc.ctypes.data, sr, out.ctypes.data)
    return out


def c_inter_encode(prev, cur, sr, scale=1.0, zigzag=False, rows=None):
    """The open-loop P-frame residual chain of ivc_oracle.inter_encode (videocodec.py:52-73:
    ME against the previous source frame, MC, residual = cur - prediction, DCT + quantise)
    with the ME from the C restatement, so that it finishes in seconds at 1080p-8K.
    rows=(by0, by1) restricts the output to those block rows (candidate validity and the
    prediction still use the whole frame).  Returns (mv [r, w, 1] int64, q [r, w, 3, 8, 8] or
    [r, w, 3, 64] int32)."""
    import numpy as np
    from . import ivc_oracle as O
    prev = np.ascontiguousarray(prev, dtype=np.uint8)
    cur = np.ascontiguousarray(cur, dtype=np.uint8)
    H, W = prev.shape
    by0, by1 = rows if rows is not None else (0, H // 8)
    mv = c_motion_vectors(prev, cur, sr, exact_u8=True, rows=(by0, by1))
    # motion.py:80-95 block copy for the selected rows (zeros where the block leaves the frame)
    n = 2 * sr + 1
    idx = mv[..., 0]
    dy, dx = idx // n - sr, idx % n - sr
    by = np.arange(by0, by1)[:, None] * 8 + dy
    bx = np.arange(W // 8)[None, :] * 8 + dx
    inside = (by >= 0) & (by + 8 <= H) & (bx >= 0) & (bx + 8 <= W)
    yy = np.clip(by, 0, H - 8)[:, :, None, None] + np.arange(8)[None, None, :, None]
    xx = np.clip(bx, 0, W - 8)[:, :, None, None] + np.arange(8)[None, None, None, :]
    blocks = prev.astype(np.float64)[yy, xx] * inside[:, :, None, None]
    pred = blocks.transpose(0, 2, 1, 3).reshape((by1 - by0) * 8, W)
    resid = cur[8 * by0:8 * by1].astype(np.float64) - pred
    return mv, O.intra_encode(resid[..., None], scale, zigzag)
