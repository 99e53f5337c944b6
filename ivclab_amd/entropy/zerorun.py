"""ZeroRunCoder on the MI355X (drop-in for ivclab/entropy/zerorun.py:4-88).

encode: zig-zag blocks [h, w, c, p] -> int32 symbol stream, computed by libivc's
wave-per-block kernels (ivc_zerorun_encode).  decode: symbol stream -> [h, w, c, block_size]
int32 blocks (ivc_zerorun_decode), raising the reference's exceptions for malformed
streams.  The reference's DEBUG prints are not reproduced.
"""
from __future__ import annotations

import numpy as np
from einops import rearrange

from .. import _native as N

_I32 = np.iinfo(np.int32)


def _as_int32_symbols(x: np.ndarray) -> np.ndarray:
    """Values as the reference emits them (int(val) into an int32 array, zerorun.py:36,40)."""
    if x.dtype == np.int32:
        return x
    if x.dtype == np.bool_ or np.issubdtype(x.dtype, np.integer):
        if x.size and (x.min() < _I32.min or x.max() > _I32.max):
            big = x.max() if x.max() > _I32.max else x.min()
            raise OverflowError(f"Python integer {int(big)} out of bounds for int32")
        return x.astype(np.int32)
    if np.issubdtype(x.dtype, np.floating):
        if np.isnan(x).any():
            raise ValueError("cannot convert float NaN to integer")
        if np.isinf(x).any():
            raise OverflowError("cannot convert float infinity to integer")
        t = np.trunc(x)
        if ((x != 0) & (t == 0)).any():
            raise NotImplementedError(
                "ZeroRunCoder: nonzero symbols with |value| < 1 (emitted by the reference as a "
                "0 value) are not supported")
        if t.size and (t.min() < _I32.min or t.max() > _I32.max):
            raise OverflowError("Python integer out of bounds for int32")
        return t.astype(np.int32)
    raise TypeError(f"ZeroRunCoder: unsupported symbol dtype {x.dtype}")


class ZeroRunCoder:
    """ivclab.entropy.zerorun.ZeroRunCoder (zerorun.py:4-8): EOB symbol and block size."""

    def __init__(self, end_of_block=4000, block_size=64):
        self.EOB = end_of_block
        self.block_size = block_size

    def encode(self, flat_patch_img):
        """zerorun.py:10-43: (h w c) blocks of the first block_size coefficients ->
        [value | 0, run]* EOB per block, one int32 stream."""
        flat = rearrange(np.asarray(flat_patch_img), "h w c p -> (h w c) p")
        nblk, p = flat.shape
        B = int(self.block_size)
        if B > p and nblk:
            raise IndexError(f"index {B - 1} is out of bounds for axis 0 with size {p}")
        if B > 64:
            raise NotImplementedError("ZeroRunCoder: block_size > 64 is not supported")
        src = np.ascontiguousarray(_as_int32_symbols(np.ascontiguousarray(flat[:, :max(B, 1)])))
        eob = int(self.EOB)
        if not _I32.min <= eob <= _I32.max:
            raise OverflowError(f"Python integer {eob} out of bounds for int32")
        cap = nblk * (B + (B + 1) // 2 + 1)
        out = np.empty(max(cap, 1), np.int32)
        nsym = np.zeros(1, np.int64)
        N.check(N.lib().ivc_zerorun_encode(N.ptr(src), nblk, src.shape[1], B, eob, N.ptr(out),
                                           cap, N.ptr(nsym)), "zerorun_encode")
        return out[:int(nsym[0])].copy()

    def decode(self, encoded, original_shape):
        """zerorun.py:46-88, errors included."""
        h, w, c = original_shape
        expected = h * w * c
        B = int(self.block_size)
        sym, is_list = decode_input(encoded)
        if expected == 0:
            # the reference rearranges an empty list: the same einops error
            return rearrange(np.array([], dtype=np.int32), "(h w c) p -> h w c p",
                             h=h, w=w, c=c, p=B)
        if B > 64:
            raise NotImplementedError("ZeroRunCoder: block_size > 64 is not supported")
        out = N.empty((expected, B), np.int32)
        err = np.zeros(3, np.int64)
        N.check(N.lib().ivc_zerorun_decode(N.ptr(sym), sym.size, expected, B, int(self.EOB),
                                           N.ptr(out), N.ptr(err)), "zerorun_decode")
        raise_stream_error(err, is_list)
        return out.reshape(h, w, c, B)


def decode_input(encoded):
    """The symbol stream as contiguous int32 (the reference reads it element by element, so
    any 1-D sequence of integers is accepted) and whether it came as a Python list (the
    reference's IndexError message differs between lists and arrays)."""
    is_list = not isinstance(encoded, np.ndarray)
    sym = np.asarray(encoded)
    if sym.ndim != 1:
        sym = sym.reshape(-1)
    if sym.size == 0:
        sym = sym.astype(np.int32)
    return np.ascontiguousarray(_as_int32_symbols(sym)), is_list


def raise_stream_error(err, is_list):
    """The reference's exception for a malformed stream (err as ivc_zerorun_decode fills it)."""
    code = int(err[0])
    if code == 1:
        raise ValueError(f"Block size exceeded: {int(err[1])}")
    if code == 2:
        raise ValueError("Unexpected end of encoded symbols")
    if code == 3:
        n = int(err[1])
        raise IndexError("list index out of range" if is_list
                         else f"index {n} is out of bounds for axis 0 with size {n}")
    if code == 4:
        raise ValueError(f"Expected {int(err[1])} blocks, got {int(err[2])}")
