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
