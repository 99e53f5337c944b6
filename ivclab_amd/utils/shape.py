"""ZigZag and Patcher — drop-in for ivclab/utils/shape.py:4-65.

ZigZag's permutation runs in libivc's gfx950 kernel (dtype preserved, any 1/2/4/8-byte
element).  Patcher is pure layout: the same einops views the reference returns (the fused
device path folds patching into its addressing instead).
"""
from __future__ import annotations

import numpy as np
from einops import EinopsError, rearrange

from .. import _native as N

# zig-zag position of each raster index (shape.py:10-19)
ZIGZAG_ORDER = np.asarray([
    0, 1, 5, 6, 14, 15, 27, 28,
    2, 4, 7, 13, 16, 26, 29, 42,
    3, 8, 12, 17, 25, 30, 41, 43,
    9, 11, 18, 24, 31, 40, 44, 53,
    10, 19, 23, 32, 39, 45, 52, 54,
    20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61,
    35, 36, 48, 49, 57, 58, 62, 63])


def _check_elem(x: np.ndarray, what: str) -> None:
    if x.dtype.hasobject or x.dtype.itemsize not in (1, 2, 4, 8):
        raise TypeError(f"ivclab_amd: {what} supports 1/2/4/8-byte elements, got {x.dtype}")


class ZigZag:
    """An object that flattens two dimensional patches according to a zigzag rule on a
    8x8 grid (reference: ivclab/utils/shape.py:4-36)."""

    def __init__(self):
        self.zigzag_order = ZIGZAG_ORDER.copy()

    def flatten(self, patched_img: np.ndarray) -> np.ndarray:
        """[h, w, c, 8, 8] -> [h, w, c, 64] with out[..., order[k]] = in[..., k] (:21-28)."""
        x = np.asarray(patched_img)
        if x.ndim != 5:
            raise EinopsError(f"Wrong shape: expected 5 dims. Received {x.ndim}-dim tensor.")
        h, w, c, p0, p1 = x.shape
        if p0 * p1 < 64:
            raise IndexError(f"index 63 is out of bounds for axis 3 with size {p0 * p1}")
        if p0 * p1 > 64:
            raise ValueError(f"shape mismatch: value array of shape {(h, w, c, p0 * p1)} could "
                             f"not be broadcast to indexing result of shape {(h, w, c, 64)}")
        _check_elem(x, "ZigZag.flatten")
        x = np.ascontiguousarray(x)
        out = N.empty((h, w, c, 64), x.dtype)
        nrow = h * w * c
        if nrow:
            N.check(N.lib().ivc_zigzag(N.ptr(x), nrow, 64, x.dtype.itemsize, 0, N.ptr(out)),
                    "ZigZag.flatten")
        return out

    def unflatten(self, unshuffled: np.ndarray) -> np.ndarray:
        """[h, w, c, >=64] -> [h, w, c, 8, 8] gathering in[..., order[k]] (:30-36)."""
        x = np.asarray(unshuffled)
        if x.ndim < 4:
            raise IndexError("too many indices for array")
        if x.ndim != 4:
            raise EinopsError(f"Wrong shape: expected 4 dims. Received {x.ndim}-dim tensor.")
        h, w, c, n = x.shape
        if n < 64:
            raise IndexError(f"index {int(ZIGZAG_ORDER[ZIGZAG_ORDER >= n][0])} is out of bounds "
                             f"for axis 3 with size {n}")
        _check_elem(x, "ZigZag.unflatten")
        x = np.ascontiguousarray(x)
        out = N.empty((h, w, c, 8, 8), x.dtype)
        nrow = h * w * c
        if nrow:
            N.check(N.lib().ivc_zigzag(N.ptr(x), nrow, n, x.dtype.itemsize, 1, N.ptr(out)),
                    "ZigZag.unflatten")
        return out


class Patcher:
    """A class to extract/merge patches from/to an image (shape.py:38-65)."""

    def __init__(self, window_size=(8, 8)):
        self.window_size = window_size

    def patch(self, img: np.ndarray) -> np.ndarray:
        """[H, W, C] -> [H/8, W/8, C, 8, 8] (a view, as einops returns)."""
        return rearrange(img, '(h p0) (w p1) c -> h w c p0 p1',
                         p0=self.window_size[0], p1=self.window_size[1])

    def unpatch(self, patched_img: np.ndarray) -> np.ndarray:
        """[H/8, W/8, C, 8, 8] -> [H, W, C]."""
        return rearrange(patched_img, 'h w c p0 p1 -> (h p0) (w p1) c',
                         p0=self.window_size[0], p1=self.window_size[1])
