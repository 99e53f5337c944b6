"""Device-resident entry points (torch tensors already in HBM), used by bench.py and the
multi-GPU path.  Thin wrappers over the *_dev functions of include/ivc.h: pointers come
from tensor.data_ptr(), work is enqueued on the given (default: current) torch stream and
nothing is synchronised.  torch is plumbing here (allocation, streams, RCCL); every byte
of the hot path is computed by libivc's kernels.
"""
from __future__ import annotations

import numpy as np

from . import _native as N


def _stream(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _dtype_code(t) -> int:
    import torch
    m = {torch.uint8: 1, torch.int8: 2, torch.int16: 4, torch.int32: 6, torch.int64: 8,
         torch.float32: 9, torch.float64: 10}
    if t.dtype not in m:
        raise TypeError(f"unsupported tensor dtype {t.dtype}")
    return m[t.dtype]


def _contig(t, name):
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    return t


def quant_table(scale=1.0) -> np.ndarray:
    """The reference's default scaled table (PatchQuant(scale).get_quantization_table())."""
    from .quantization import PatchQuant
    return N.table_arg(PatchQuant(scale).get_quantization_table())


def intra_encode(img, table, out, zigzag=False, hist=None, hist_lo=0, stream=None):
    """img [F, H, W, C] (uint8/float32/float64) -> out [F, H/8, W/8, 3, 64] int32:
    quantize(DCT(patch(img))) (+ zig-zag); optional int64 histogram accumulated in `hist`."""
    _contig(img, "img"); _contig(out, "out")
    F, H, W, C = img.shape
    t = N.table_arg(table)
    # NumPy result type of (DCT output) / table: float32 only for float32 images and tables
    tdt = np.asarray(table).dtype
    calc = N.F32 if (_dtype_code(img) == N.F32 and tdt == np.float32) else N.F64
    hp, nb = (0, 0)
    if hist is not None:
        _contig(hist, "hist")
        hp, nb = hist.data_ptr(), hist.numel()
    N.check(N.lib().ivc_intra_encode_dev(img.data_ptr(), _dtype_code(img), F, H, W, C, N.ptr(t),
                                         calc, int(bool(zigzag)), out.data_ptr(), hp or None,
                                         hist_lo, nb, _stream(stream)), "intra_encode")


def inter_encode(frames, sr, table, mv, out, zigzag=False, stream=None, hist=None, hist_lo=0):
    """frames [F, H, W] uint8 -> mv [F-1, H/8, W/8] int64 and out [F-1, H/8, W/8, 3, 64]:
    ME(frames[f-1], frames[f]) (exact SSD) -> MC -> residual -> DCT -> quantize.  hist
    (optional, int64 [n]): the output's histogram is accumulated onto hist[clamp(v - hist_lo,
    0, n - 1)] by the encoder itself (no pass over out)."""
    for t_, n in ((frames, "frames"), (mv, "mv"), (out, "out")):
        _contig(t_, n)
    F, H, W = frames.shape
    t = N.table_arg(table)
    if hist is not None:
        import torch
        _contig(hist, "hist")
        if hist.dtype != torch.int64 or hist.numel() < 1:
            raise ValueError("inter_encode: hist must be a non-empty int64 tensor")
        N.check(N.lib().ivc_inter_encode_hist_dev(frames.data_ptr(), F, H, W, int(sr), N.ptr(t),
                                                  N.F64, int(bool(zigzag)), mv.data_ptr(),
                                                  out.data_ptr(), hist.data_ptr(), int(hist_lo),
                                                  hist.numel(), _stream(stream)), "inter_encode")
        return
    N.check(N.lib().ivc_inter_encode_dev(frames.data_ptr(), F, H, W, int(sr), N.ptr(t), N.F64,
                                         int(bool(zigzag)), mv.data_ptr(), out.data_ptr(),
                                         _stream(stream)), "inter_encode")


def motion_estimate(ref, cur, sr, mv, exact_u8=False, stream=None):
    """ref/cur [F, H, W] -> mv [F, H/8, W/8] int64 (motion.py:8-58 semantics)."""
    _contig(ref, "ref"); _contig(cur, "cur"); _contig(mv, "mv")
    F, H, W = ref.shape
    N.check(N.lib().ivc_motion_estimate_dev(ref.data_ptr(), cur.data_ptr(), _dtype_code(ref), F,
                                            H, W, int(sr), N.ME_EXACT_U8 if exact_u8 else N.ME_NUMPY,
                                            mv.data_ptr(), _stream(stream)), "motion_estimate")


def histogram(sym, lo, hist, stream=None):
    """hist[v - lo] += 1 over the int32 or int64 tensor sym (clamped into the end bins);
    hist is an int64 tensor of nbins counts (accumulated onto)."""
    import torch
    _contig(sym, "sym"); _contig(hist, "hist")
    if hist.dtype != torch.int64:
        raise ValueError("histogram: hist must be int64")
    if sym.dtype == torch.int32:
        fn = N.lib().ivc_histogram_i32_dev
    elif sym.dtype == torch.int64:
        fn = N.lib().ivc_histogram_i64_dev
    else:
        raise ValueError(f"histogram: symbols must be int32 or int64, got {sym.dtype}")
    N.check(fn(sym.data_ptr(), sym.numel(), int(lo), hist.numel(), hist.data_ptr(),
               _stream(stream)), "histogram")


def zerorun_encode(blocks, offsets, out, block_size=64, eob=4000, stream=None):
    """blocks [..., p] int32 (zig-zag rows, (h w c) order) -> offsets [nblk + 1] int64
    (offsets[nblk] = stream length) and the symbols in out (int32, written up to its
    length).  Asynchronous: read offsets[-1] after the stream to size or check out."""
    import torch
    _contig(blocks, "blocks"); _contig(offsets, "offsets"); _contig(out, "out")
    if blocks.dtype != torch.int32 or offsets.dtype != torch.int64 or out.dtype != torch.int32:
        raise ValueError("zerorun_encode: blocks/out must be int32 and offsets int64")
    p = blocks.shape[-1]
    nblk = blocks.numel() // p if p else 0
    if offsets.numel() < nblk + 1:
        raise ValueError("zerorun_encode: offsets needs nblk + 1 entries")
    N.check(N.lib().ivc_zerorun_encode_dev(blocks.data_ptr(), nblk, p, int(block_size), int(eob),
                                           offsets.data_ptr(), out.data_ptr(), out.numel(),
                                           _stream(stream)), "zerorun_encode")


def zerorun_decode(sym, nblk, out, err, block_size=64, eob=4000, stream=None):
    """sym [n] int32 -> out [nblk, block_size] int32; err [3] int64 receives the stream's
    verdict (0 = decoded; see include/ivc.h).  Asynchronous."""
    import torch
    _contig(sym, "sym"); _contig(out, "out"); _contig(err, "err")
    if sym.dtype != torch.int32 or out.dtype != torch.int32 or err.dtype != torch.int64:
        raise ValueError("zerorun_decode: sym/out must be int32 and err int64")
    if out.numel() < nblk * block_size or err.numel() < 3:
        raise ValueError("zerorun_decode: out needs nblk * block_size entries, err 3")
    N.check(N.lib().ivc_zerorun_decode_dev(sym.data_ptr(), sym.numel(), int(nblk), int(block_size),
                                           int(eob), out.data_ptr(), err.data_ptr(),
                                           _stream(stream)), "zerorun_decode")


def minmax(sym, mm, stream=None):
    """mm[0], mm[1] = min, max of the int32 tensor sym (int32 mm of 2)."""
    import torch
    _contig(sym, "sym"); _contig(mm, "mm")
    if sym.dtype != torch.int32 or mm.dtype != torch.int32 or mm.numel() < 2:
        raise ValueError("minmax: int32 symbols and an int32 output of 2")
    N.check(N.lib().ivc_minmax_i32_dev(sym.data_ptr(), sym.numel(), mm.data_ptr(),
                                       _stream(stream)), "minmax")


def intra_symbols(frames, table, out, nsym, eob=4000, stream=None, hist=None, hist_lo=0):
    """u8 frames [F, H, W] or [F, H, W, C] -> the zero-run symbol stream of their quantised
    zig-zag blocks (IntraCodec.image2symbols without colour conversion, one fused pass per
    frame batch; the coefficients never reach memory).  out: int32 (written up to its
    length), nsym: int64 device scalar receiving the stream length.  hist (optional, int64
    [n]): the emitted stream's histogram is accumulated onto hist[clamp(v - hist_lo, 0,
    n - 1)] by the emission pass itself.  Asynchronous."""
    import torch
    _contig(frames, "frames"); _contig(out, "out"); _contig(nsym, "nsym")
    if frames.dtype != torch.uint8 or out.dtype != torch.int32 or nsym.dtype != torch.int64:
        raise ValueError("intra_symbols: uint8 frames, int32 out, int64 nsym")
    F, H, W = frames.shape[:3]
    C = frames.shape[3] if frames.dim() == 4 else 1
    t = N.table_arg(table)
    if hist is None:
        N.check(N.lib().ivc_intra_symbols_dev(frames.data_ptr(), N.DTYPE_CODE[np.dtype(np.uint8)], F,
                                              H, W, C, N.ptr(t), int(eob), out.data_ptr(),
                                              out.numel(), nsym.data_ptr(), _stream(stream)),
                "intra_symbols")
        return
    _contig(hist, "hist")
    if hist.dtype != torch.int64 or hist.dim() != 1 or hist.numel() < 1:
        raise ValueError("intra_symbols: hist must be a 1-D int64 tensor")
    if not -(1 << 31) <= int(hist_lo) < (1 << 31) or hist.numel() >= (1 << 31):
        raise ValueError("intra_symbols: hist_lo / hist size out of int32 range")
    N.check(N.lib().ivc_intra_symbols_hist_dev(frames.data_ptr(), N.DTYPE_CODE[np.dtype(np.uint8)], F,
                                               H, W, C, N.ptr(t), int(eob), out.data_ptr(),
                                               out.numel(), nsym.data_ptr(), hist.data_ptr(),
                                               int(hist_lo), hist.numel(), _stream(stream)),
            "intra_symbols")


def intra_decode_image(q, table, out, unzigzag=True, to_rgb=False, stream=None):
    """q [F, h, w, C, 64] int32 (C = 1 or 3) -> out [F, 8h, 8w, 3] float64: the unpatched
    DCT.inverse_transform(PatchQuant.dequantize(ZigZag.unflatten(q))) (C = 1 broadcasts over
    the 3 table planes), optionally through ycbcr2rgb.  Asynchronous."""
    import torch
    _contig(q, "q"); _contig(out, "out")
    if q.dtype != torch.int32 or out.dtype != torch.float64 or q.dim() != 5 or q.shape[-1] != 64:
        raise ValueError("intra_decode_image: q [F, h, w, C, 64] int32, out float64")
    F, h, w, C, _ = q.shape
    if tuple(out.shape) != (F, 8 * h, 8 * w, 3):
        raise ValueError(f"intra_decode_image: out must be {(F, 8 * h, 8 * w, 3)}")
    t = N.table_arg(table)
    N.check(N.lib().ivc_intra_decode_image_dev(q.data_ptr(), F, 8 * h, 8 * w, C, N.ptr(t),
                                               int(bool(unzigzag)), int(bool(to_rgb)),
                                               out.data_ptr(), _stream(stream)), "intra_decode_image")


def symbols2image(sym, C, table, out, err, eob=4000, to_rgb=False, stream=None):
    """IntraCodec.symbols2image on the device: the int32 zero-run stream of F frames of
    [h, w, C] blocks -> out [F, 8h, 8w, 3] float64 (zero-run decode -> un-zig-zag ->
    dequantise -> IDCT -> unpatch, optionally ycbcr2rgb).  err [3] int64 receives the
    stream's verdict as zerorun_decode's.  Asynchronous."""
    import torch
    _contig(sym, "sym"); _contig(out, "out"); _contig(err, "err")
    if sym.dtype != torch.int32 or out.dtype != torch.float64 or err.dtype != torch.int64:
        raise ValueError("symbols2image: int32 sym, float64 out, int64 err")
    if sym.dim() != 1 or err.dim() != 1 or err.numel() < 3:
        raise ValueError("symbols2image: sym must be 1-D, err must hold 3 values")
    if out.dim() != 4 or out.shape[3] != 3 or out.shape[1] % 8 or out.shape[2] % 8:
        raise ValueError("symbols2image: out must be [F, 8h, 8w, 3] (the kernel writes 3 planes)")
    if int(C) not in (1, 3):
        raise ValueError("symbols2image: C must be 1 or 3")
    F, H, W, _ = out.shape
    t = N.table_arg(table)
    N.check(N.lib().ivc_symbols2image_dev(sym.data_ptr(), sym.numel(), F, H, W, int(C), N.ptr(t),
                                          int(eob), int(bool(to_rgb)), out.data_ptr(),
                                          err.data_ptr(), _stream(stream)), "symbols2image")


def intra_encode_luma(frames, table, out, zigzag=False, stream=None):
    """u8 frames [F, H, W] (or [F, H, W, 1]) -> out [F, H/8, W/8, 64] int32: plane 0 (the
    luminance table) of intra_encode's output.  Not the reference's output (PatchQuant
    broadcasts C = 1 to 3 planes, patchquant.py:59): a reported 5 B/px variant."""
    import torch
    _contig(frames, "frames"); _contig(out, "out")
    if frames.dtype != torch.uint8 or out.dtype != torch.int32:
        raise ValueError("intra_encode_luma: uint8 frames, int32 out")
    if frames.dim() == 4 and frames.shape[3] != 1:
        raise ValueError("intra_encode_luma: one channel")
    F, H, W = frames.shape[:3]
    if tuple(out.shape) != (F, H // 8, W // 8, 64):
        raise ValueError(f"intra_encode_luma: out must be {(F, H // 8, W // 8, 64)}")
    t = N.table_arg(table)
    N.check(N.lib().ivc_intra_encode_luma_dev(frames.data_ptr(), F, H, W, N.ptr(t),
                                              int(bool(zigzag)), out.data_ptr(), _stream(stream)),
            "intra_encode_luma")
