"""DiscreteCosineTransform — drop-in for ivclab/signal/dct.py:4-46.

Same constructor, attribute and methods; the 2-D DCT-II / DCT-III of every trailing 8x8
block runs in libivc's gfx950 kernel, which reproduces scipy.fft's pocketfft op sequence
bit for bit (dtype rules as scipy: float32 -> float32, other real dtypes -> float64).
"""
from __future__ import annotations

import numpy as np

from .. import _native as N


def patch_view_image(x):
    """If x is Patcher.patch's view of a C-contiguous [H, W, C] image (shape.py:45-54:
    [H/8, W/8, C, 8, 8] with strides (8 W C, 8 C, 1, W C, C) elements), that image as an
    [H, W, C] array over the same memory; else None."""
    if x.ndim != 5 or x.shape[-2:] != (8, 8) or x.flags.c_contiguous:
        return None
    h, w, C = x.shape[:3]
    s = x.itemsize
    W = 8 * w
    if x.strides != (8 * W * C * s, 8 * C * s, s, W * C * s, C * s):
        return None
    return np.lib.stride_tricks.as_strided(x, shape=(8 * h, W, C), strides=(W * C * s, C * s, s))


_F64 = np.dtype(np.float64)
_F32 = np.dtype(np.float32)


def dct2d(a, norm="ortho", inverse=False) -> np.ndarray:
    """dct (or idct) along axis -1 then axis -2 of every trailing 8x8 block of `a`."""
    # fast path for small arrays of a supported dtype (the reference's per-block loops call
    # this once per (8, 8) block: the general checks below cost more than the GPU round trip's
    # host side): C-contiguous ones in one C step (ivc_pyfast.c), others through ctypes
    if type(a) is np.ndarray and a.size <= 4096:
        F = N.fast()
        nc = N.NORM_CODE.get(norm)
        if F is not None and nc is not None:
            r = F.dct8x8(a, nc, 1 if inverse else 0)
            if r is not None:
                if type(r) is int:
                    N.check(r, "DiscreteCosineTransform")
                return r
    if type(a) is np.ndarray and a.shape[-2:] == (8, 8) and 0 < a.size <= 4096:
        code = N.DTYPE_CODE.get(a.dtype)
        nc = N.NORM_CODE.get(norm)
        if code is not None and nc is not None:
            if not a.flags.c_contiguous:        # e.g. one channel of a patch view: a 512 B copy
                a = np.ascontiguousarray(a)
            od = _F32 if code == N.F32 else _F64
            out = np.empty(a.shape, od)
            N.check(N.lib().ivc_dct8x8(N.ptr(a), code, a.size // 64, N.ptr(out),
                                       N.F32 if od is _F32 else N.F64,
                                       1 if inverse else 0, nc), "DiscreteCosineTransform")
            return out
    if norm not in N.NORM_CODE:
        raise ValueError(f'Invalid norm value {norm!r}, should be "backward", "ortho" or "forward"')
    x = np.asarray(a)
    if np.iscomplexobj(x):  # scipy transforms the real and imaginary parts separately
        re = dct2d(x.real, norm, inverse)
        return re + 1j * dct2d(x.imag, norm, inverse)
    if x.ndim < 2:
        raise np.exceptions.AxisError(-2, x.ndim)
    if x.shape[-1] < 1 or x.shape[-2] < 1:
        raise ValueError(f"invalid number of data points ({min(x.shape[-2:])}) specified")
    if x.shape[-2:] != (8, 8):
        raise NotImplementedError(
            f"ivclab_amd: DCT is implemented for 8x8 blocks (the codec block size); got {x.shape[-2:]}")
    if not x.dtype.isnative:
        x = x.astype(x.dtype.newbyteorder("="))   # same values in the host byte order
    if x.dtype == np.float16:
        x = x.astype(np.float32)          # scipy's _asfarray does the same
    elif x.dtype == np.bool_:
        x = x.view(np.uint8)
    if x.dtype not in N.DTYPE_CODE:
        raise TypeError(f"ivclab_amd: unsupported dtype {x.dtype} for the DCT")
    out_dtype = np.float32 if x.dtype == np.float32 else np.float64
    out = N.empty(x.shape, out_dtype)
    nblk = x.size // 64
    if nblk == 0:
        return out
    L = N.lib()
    img = patch_view_image(x)
    if img is not None:          # transform(patch(img)): the kernel reads the image in place
        N.check(L.ivc_dct8x8_image(N.ptr(img), N.DTYPE_CODE[img.dtype], img.shape[0], img.shape[1],
                                   img.shape[2], N.ptr(out), N.DTYPE_CODE[np.dtype(out_dtype)],
                                   1 if inverse else 0, N.NORM_CODE[norm]), "DiscreteCosineTransform")
        return out
    x = np.ascontiguousarray(x)
    N.check(L.ivc_dct8x8(N.ptr(x), N.DTYPE_CODE[x.dtype], nblk, N.ptr(out),
                         N.DTYPE_CODE[np.dtype(out_dtype)], 1 if inverse else 0,
                         N.NORM_CODE[norm]), "DiscreteCosineTransform")
    return out


class DiscreteCosineTransform:
    """A class to implement the forward and inverse transform of the DCT Type II
    (reference: ivclab/signal/dct.py:4-46)."""

    def __init__(self, norm="ortho"):
        self.norm = norm

    def transform(self, patched_img: np.ndarray) -> np.ndarray:
        """DCT-II along the last axis, then the second-to-last (dct.py:12-28)."""
        return dct2d(patched_img, self.norm, inverse=False)

    def inverse_transform(self, transformed: np.ndarray) -> np.ndarray:
        """DCT-III along the last axis, then the second-to-last (dct.py:30-46)."""
        return dct2d(transformed, self.norm, inverse=True)
