"""zigzag_scan — drop-in for ivclab/signal/zigzag.py:3-26 (one 8x8 block -> (64,))."""
from __future__ import annotations

import numpy as np

from .. import _native as N


def zigzag_scan(block):
    """Perform zig-zag scan on an 8x8 block (zigzag.py:3-26)."""
    assert block.shape == (8, 8), "Input must be an 8x8 block"
    x = np.ascontiguousarray(block)
    if x.dtype.itemsize not in (1, 2, 4, 8) or x.dtype.hasobject:
        raise TypeError(f"ivclab_amd: unsupported dtype {x.dtype} for zigzag_scan")
    out = np.empty(64, dtype=x.dtype)
    N.check(N.lib().ivc_zigzag(N.ptr(x), 1, 64, x.dtype.itemsize, 0, N.ptr(out)), "zigzag_scan")
    return out
