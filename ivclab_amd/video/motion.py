"""MotionCompensator — drop-in for ivclab/video/motion.py:3-97.

compute_motion_vector runs the full search in libivc's gfx950 kernel with the reference's
exact SSD arithmetic for the input dtype (NumPy wrap-around for integer dtypes, NumPy's
pairwise summation for float dtypes) and its first-strict-minimum tie-break;
reconstruct_with_motion_vector is the block-copy kernel (zeros where the displaced block
leaves the frame).
"""
from __future__ import annotations

import numpy as np

from .. import _native as N


def _me_dtype(ref: np.ndarray, cur: np.ndarray) -> np.dtype:
    dt = np.result_type(ref.dtype, cur.dtype)
    if dt == np.bool_:
        raise TypeError("numpy boolean subtract, the `-` operator, is not supported")
    if dt not in N.DTYPE_CODE:
        raise TypeError(f"ivclab_amd: motion estimation on {dt} is not supported")
    return dt


class MotionCompensator:

    def __init__(self, search_range=4):
        self.search_range = search_range

    def compute_motion_vector(self, ref_image, image):
        """Per 8x8 block of `image`, the displacement index (dy+sr)*(2sr+1)+(dx+sr) of the
        SSD-closest window of `ref_image` (motion.py:8-58).  Returns [H/8, W/8, 1] int64."""
        ref, cur = np.asarray(ref_image), np.asarray(image)
        H, W = ref.shape
        sr = int(self.search_range)
        if sr < 0:
            raise ValueError("search_range must be non-negative")
        if cur.shape != ref.shape:
            raise ValueError(f"image shape {cur.shape} does not match reference {ref.shape}")
        if H % 8 or W % 8:
            raise ValueError(f"frame {H}x{W}: height and width must be multiples of the 8x8 block")
        dt = _me_dtype(ref, cur)
        ref = np.ascontiguousarray(ref, dtype=dt)
        cur = np.ascontiguousarray(cur, dtype=dt)
        mv = np.empty((H // 8, W // 8, 1), dtype=np.int64)
        if mv.size:
            N.check(N.lib().ivc_motion_estimate(N.ptr(ref), N.ptr(cur), N.DTYPE_CODE[dt], 1, H, W,
                                                sr, N.ME_NUMPY, N.ptr(mv)),
                    "MotionCompensator.compute_motion_vector")
        return mv

    def reconstruct_with_motion_vector(self, ref_image, motion_vector):
        """Block-copy prediction [H, W, C] from ref_image and the motion indices
        (motion.py:60-97); blocks whose displaced window leaves the frame stay zero."""
        ref = np.asarray(ref_image)
        H, W, C = ref.shape
        sr = int(self.search_range)
        if sr < 0:
            raise ValueError("search_range must be non-negative")
        if H % 8 or W % 8:
            raise ValueError(f"frame {H}x{W}: height and width must be multiples of the 8x8 block")
        mv = np.asarray(motion_vector)
        h, w = H // 8, W // 8
        if mv.ndim != 3 or mv.shape[0] < h or mv.shape[1] < w or mv.shape[2] < 1:
            raise IndexError(f"motion vector of shape {mv.shape} does not cover {h}x{w} blocks")
        if not np.issubdtype(mv.dtype, np.integer):
            raise TypeError("slice indices must be integers")
        if ref.dtype.hasobject or ref.dtype.itemsize not in (1, 2, 4, 8):
            raise TypeError(f"ivclab_amd: unsupported dtype {ref.dtype} for motion compensation")
        mvc = np.ascontiguousarray(mv[:h, :w, 0], dtype=np.int64)
        ref = np.ascontiguousarray(ref)
        out = N.empty_like(ref)
        if out.size:
            N.check(N.lib().ivc_motion_compensate(N.ptr(ref), ref.dtype.itemsize, 1, H, W, C,
                                                  N.ptr(mvc), sr, N.ptr(out)),
                    "MotionCompensator.reconstruct_with_motion_vector")
        return out
