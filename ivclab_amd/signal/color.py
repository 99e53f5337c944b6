"""Colour conversions on the MI355X (drop-in for ivclab/signal/color.py:3-63).

rgb2ycbcr reproduces NumPy's `image @ M.T + offset` bit for bit (OpenBLAS dgemm's k-order
fused multiply-adds, ivc_color.hip); ycbcr2rgb and rgb2gray restate the reference's
elementwise expressions in its evaluation order and result dtypes.  New arrays are
returned; inputs are never modified.
"""
from __future__ import annotations

import numpy as np

from .. import _native as N

_M = np.array([[0.299, 0.587, 0.114], [-0.168736, -0.331264, 0.5], [0.5, -0.418688, -0.081312]])


def _kernel_input(a: np.ndarray, what: str) -> np.ndarray:
    if a.dtype == np.bool_:
        return a.astype(np.uint8)
    if a.dtype == np.float16:
        raise NotImplementedError(f"{what}: float16 images are not supported")
    if a.dtype not in N.DTYPE_CODE:
        raise NotImplementedError(f"{what}: dtype {a.dtype} is not supported")
    return np.ascontiguousarray(a)


def rgb2gray(image: np.array):
    """color.py:3-13: np.mean(image, axis=-1, keepdims=True)."""
    a = np.asarray(image)
    if a.ndim == 0:
        raise np.exceptions.AxisError("axis -1 is out of bounds for array of dimension 0")
    C = a.shape[-1]
    if C == 0 or C >= 8:
        raise NotImplementedError("rgb2gray: 1 to 7 channels are supported")
    x = _kernel_input(a, "rgb2gray")
    out = N.empty(a.shape[:-1] + (1,), np.float32 if x.dtype == np.float32 else np.float64)
    npix = x.size // C
    N.check(N.lib().ivc_rgb2gray(N.ptr(x), N.DTYPE_CODE[x.dtype], npix, C, N.ptr(out)), "rgb2gray")
    return out


def rgb2ycbcr(image: np.array):
    """color.py:15-38: image @ M.T + [0, 128, 128] (BT.601), float64."""
    a = np.asarray(image)
    if a.ndim == 0 or a.shape[-1] != 3:
        np.matmul(np.zeros(a.shape[-1:] if a.ndim else (), a.dtype), _M.T)   # NumPy's own error
    x = _kernel_input(a, "rgb2ycbcr")
    out = N.empty(a.shape, np.float64)
    N.check(N.lib().ivc_rgb2ycbcr(N.ptr(x), N.DTYPE_CODE[x.dtype], x.size // 3, N.ptr(out)),
            "rgb2ycbcr")
    return out


def ycbcr2rgb(image: np.array):
    """color.py:40-63: R = Y + 1.402 Cr, G = Y - 0.344136 Cb - 0.714136 Cr, B = Y + 1.772 Cb
    (Cb, Cr offset by 128), clipped to [0, 255]; float32 stays float32."""
    a = np.asarray(image)
    if a.ndim != 3:
        a[:, :, 0]                                                   # NumPy's own IndexError
        raise IndexError("ycbcr2rgb: [H, W, C] input expected")
    if a.shape[2] < 3:
        a[:, :, 2]
    x = _kernel_input(a, "ycbcr2rgb")
    out = N.empty(a.shape[:2] + (3,), np.float32 if x.dtype == np.float32 else np.float64)
    N.check(N.lib().ivc_ycbcr2rgb(N.ptr(x), N.DTYPE_CODE[x.dtype], a.shape[0] * a.shape[1],
                                  a.shape[2], N.ptr(out)), "ycbcr2rgb")
    return out
