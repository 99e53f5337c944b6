"""NumPy/SciPy restatement of the ivclab hot path — TEST INFRASTRUCTURE ONLY (see __init__).

Every function states the reference behaviour it restates (file:line under
/root/reference, snapshot 2025-06-29).  The arithmetic deliberately goes through the same
library calls the reference makes (scipy.fft.dct/idct -> pocketfft, np.round, NumPy
broadcasting and casting), so that the results are the reference's results on the same
inputs.  Parity of this module with the reference itself is pinned by the committed golden
vectors (tests/golden/*.npz, tests/test_oracle_golden.py).
"""
from __future__ import annotations

import numpy as np
import scipy.fft as _sfft

# ---------------------------------------------------------------- tables ----------------
# ivclab/quantization/patchquant.py:16-25 (luminance) and :28-37 (chrominance), float32
LUMINANCE = np.array(
    [[16, 11, 10, 16, 24, 40, 51, 61], [12, 12, 14, 19, 26, 58, 60, 55],
     [14, 13, 16, 24, 40, 57, 69, 56], [14, 17, 22, 29, 51, 87, 80, 62],
     [18, 55, 37, 56, 68, 109, 103, 77], [24, 35, 55, 64, 81, 104, 113, 92],
     [49, 64, 78, 87, 103, 121, 120, 101], [72, 92, 95, 98, 112, 100, 103, 99]],
    dtype=np.float32)
CHROMINANCE = np.full((8, 8), 99, dtype=np.float32)
CHROMINANCE[:4, :4] = [[17, 18, 24, 47], [18, 21, 26, 66], [24, 13, 56, 99], [47, 66, 99, 99]]

# ivclab/utils/shape.py:10-19: zig-zag position of each raster index
ZZ_ORDER = np.array([
    0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42,
    3, 8, 12, 17, 25, 30, 41, 43, 9, 11, 18, 24, 31, 40, 44, 53,
    10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63])
# ivclab/signal/zigzag.py:15-24 as raster indices (the inverse permutation of ZZ_ORDER)
ZZ_SCAN = np.argsort(ZZ_ORDER)


# ---------------------------------------------------------------- DCT -------------------
def dct_transform(a, norm="ortho"):
    """DiscreteCosineTransform.transform (ivclab/signal/dct.py:12-28): dct along axis -1,
    then along axis -2, scipy type-II with the given norm."""
    return _sfft.dct(_sfft.dct(a, axis=-1, norm=norm), axis=-2, norm=norm)


def dct_inverse(a, norm="ortho"):
    """DiscreteCosineTransform.inverse_transform (ivclab/signal/dct.py:30-46)."""
    return _sfft.idct(_sfft.idct(a, axis=-1, norm=norm), axis=-2, norm=norm)


# ---------------------------------------------------------------- quantisation ----------
def quant_table(scale=1.0, luminance=None, chrominance=None):
    """PatchQuant.get_quantization_table (patchquant.py:39-42): stack(lum, chrom, chrom) *
    scale, keeping NumPy's dtype result (float32 for a Python-float scale)."""
    lum = LUMINANCE if luminance is None else luminance
    chrom = CHROMINANCE if chrominance is None else chrominance
    return np.stack([lum, chrom, chrom], axis=0) * scale


def quantize(x, scale=1.0, luminance=None, chrominance=None):
    """PatchQuant.quantize (patchquant.py:44-60): round-half-even of x / table broadcast
    as [1,1,3,8,8], cast to int32."""
    t = quant_table(scale, luminance, chrominance)
    return np.round(x / t[None, None]).astype(np.int32)


def dequantize(q, scale=1.0, luminance=None, chrominance=None):
    """PatchQuant.dequantize (patchquant.py:62-78): q * table, cast (truncating) to int32."""
    t = quant_table(scale, luminance, chrominance)
    return (q * t[None, None]).astype(np.int32)


# ---------------------------------------------------------------- layout ----------------
def patch(img, window=(8, 8)):
    """Patcher.patch (ivclab/utils/shape.py:45-54): [H,W,C] -> [H/8, W/8, C, 8, 8] view."""
    H, W, C = img.shape
    p0, p1 = window
    return img.reshape(H // p0, p0, W // p1, p1, C).transpose(0, 2, 4, 1, 3)


def unpatch(blocks, window=(8, 8)):
    """Patcher.unpatch (shape.py:56-65): [h, w, C, 8, 8] -> [h*8, w*8, C]."""
    h, w, C, p0, p1 = blocks.shape
    return blocks.transpose(0, 3, 1, 4, 2).reshape(h * p0, w * p1, C)


def zigzag_flatten(x):
    """ZigZag.flatten (shape.py:21-28): [h,w,c,8,8] -> [h,w,c,64], out[..., ZZ_ORDER[k]] =
    in[..., k]; dtype preserved."""
    h, w, c, p0, p1 = x.shape
    flat = x.reshape(h, w, c, p0 * p1)
    out = np.zeros_like(flat)
    out[:, :, :, ZZ_ORDER] = flat
    return out


def zigzag_unflatten(x):
    """ZigZag.unflatten (shape.py:30-36): gather by ZZ_ORDER, then [h,w,c,8,8]."""
    h, w, c, _ = x.shape
    return x[:, :, :, ZZ_ORDER].reshape(h, w, c, 8, 8)


def zigzag_scan(block):
    """zigzag_scan (ivclab/signal/zigzag.py:3-26): one 8x8 block -> (64,) in scan order."""
    assert block.shape == (8, 8), "Input must be an 8x8 block"
    return np.array([block[k // 8, k % 8] for k in ZZ_SCAN])


# ---------------------------------------------------------------- motion ----------------
def motion_vectors_loop(ref, cur, sr):
    """MotionCompensator.compute_motion_vector (ivclab/video/motion.py:8-58), the literal
    per-block / per-candidate loop: candidates from `ref`, blocks from `cur`, dy outer and
    dx inner over [-sr, sr], out-of-frame candidates skipped, SSD = np.sum((blk-cand)**2)
    in the input dtype, first strict minimum wins, index (dy+sr)(2sr+1)+(dx+sr).
    Slow (one np.sum per candidate): small frames and the CPU baseline sample only."""
    H, W = ref.shape
    n = 2 * sr + 1
    mv = np.zeros((H // 8, W // 8, 1), dtype=int)
    for by in range(H // 8):
        for bx in range(W // 8):
            y, x = 8 * by, 8 * bx
            blk = cur[y:y + 8, x:x + 8]
            best, bdy, bdx = float("inf"), 0, 0
            for dy in range(-sr, sr + 1):
                if y + dy < 0 or y + dy + 8 > H:
                    continue
                for dx in range(-sr, sr + 1):
                    if x + dx < 0 or x + dx + 8 > W:
                        continue
                    s = np.sum((blk - ref[y + dy:y + dy + 8, x + dx:x + dx + 8]) ** 2)
                    if s < best:
                        best, bdy, bdx = s, dy, dx
            mv[by, bx, 0] = (bdy + sr) * n + (bdx + sr)
    return mv


def _pairwise64(sq):
    """np.sum over a contiguous 8x8 float block, in NumPy's pairwise order for n = 64:
    eight column accumulators summed down the rows, then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))."""
    r = sq[..., 0, :].copy()
    for u in range(1, 8):
        r = r + sq[..., u, :]
    return ((r[..., 0] + r[..., 1]) + (r[..., 2] + r[..., 3])) + \
           ((r[..., 4] + r[..., 5]) + (r[..., 6] + r[..., 7]))


def motion_vectors(ref, cur, sr):
    """Vectorised restatement of motion_vectors_loop: same candidates, same per-candidate
    arithmetic (dtype-wrapping integer sub/square with an exact wide sum; pairwise float
    sums), same first-strict-minimum rule; iterates candidates in raster order and all
    blocks at once."""
    H, W = ref.shape
    h, w = H // 8, W // 8
    n = 2 * sr + 1
    blocks = cur[:h * 8, :w * 8].reshape(h, 8, w, 8).transpose(0, 2, 1, 3)
    is_float = np.issubdtype(np.result_type(ref.dtype, cur.dtype), np.floating)
    best = None
    have = np.zeros((h, w), dtype=bool)
    bidx = np.full((h, w), sr * n + sr, dtype=np.int64)
    by = np.arange(h)[:, None] * 8
    bx = np.arange(w)[None, :] * 8
    pad = sr
    refp = np.zeros((H + 2 * pad, W + 2 * pad), dtype=ref.dtype)
    refp[pad:pad + H, pad:pad + W] = ref
    for dy in range(-sr, sr + 1):
        vy = (by + dy >= 0) & (by + dy + 8 <= H)
        for dx in range(-sr, sr + 1):
            valid = vy & (bx + dx >= 0) & (bx + dx + 8 <= W)
            if not valid.any():
                continue
            sub = refp[pad + dy:pad + dy + h * 8, pad + dx:pad + dx + w * 8]
            cand = sub.reshape(h, 8, w, 8).transpose(0, 2, 1, 3)
            sq = (blocks - cand) ** 2
            if is_float:
                s = _pairwise64(sq)
                if best is None:
                    best = np.full((h, w), np.inf, dtype=s.dtype)
                better = valid & (s < best)
            else:
                s = np.sum(sq, axis=(-2, -1))
                if best is None:
                    best = np.zeros((h, w), dtype=s.dtype)
                better = valid & (~have | (s < best))
                have |= better
            best = np.where(better, s, best)
            bidx = np.where(better, (dy + sr) * n + (dx + sr), bidx)
    return bidx[..., None].astype(int)


def motion_compensate(ref, mv, sr):
    """MotionCompensator.reconstruct_with_motion_vector (motion.py:60-97): block copy from
    the displaced position, zeros where the displaced block leaves the frame; output
    dtype = ref dtype."""
    H, W, C = ref.shape
    n = 2 * sr + 1
    out = np.zeros_like(ref)
    for by in range(H // 8):
        for bx in range(W // 8):
            idx = mv[by, bx, 0]
            dy, dx = idx // n - sr, idx % n - sr
            y, x = 8 * by + dy, 8 * bx + dx
            if y < 0 or y + 8 > H or x < 0 or x + 8 > W:
                continue
            out[8 * by:8 * by + 8, 8 * bx:8 * bx + 8, :] = ref[y:y + 8, x:x + 8, :]
    return out


# ---------------------------------------------------------------- pipelines -------------
def intra_encode(img, scale=1.0, zigzag=False):
    """quantize(dct(patch(img))) (+ zig-zag): the hot part of IntraCodec.image2symbols
    (ivclab/image/intracodec.py:66-75) for an [H,W,C] image with H, W multiples of 8."""
    q = quantize(dct_transform(patch(img)), scale)
    return zigzag_flatten(q) if zigzag else q


def intra_decode(q, scale=1.0, unzigzag=False):
    """dct_inverse(dequantize(unflatten(q))): hot part of IntraCodec.symbols2image
    (intracodec.py:115-121)."""
    if unzigzag:
        q = zigzag_unflatten(q)
    return dct_inverse(dequantize(q, scale))


def inter_encode(prev, cur, sr, scale=1.0, zigzag=False):
    """Open-loop P-frame residual path of VideoCodec.encode_decode (videocodec.py:52-73)
    with ME against the previous SOURCE frame: frames are uint8 luma, ME/MC run on the
    float64 frames (integer valued), residual = cur - prediction, then DCT + quantisation."""
    r64, c64 = prev.astype(np.float64), cur.astype(np.float64)
    mv = motion_vectors(r64, c64, sr)
    pred = motion_compensate(r64[..., None], mv, sr)[..., 0]
    resid = c64 - pred
    return mv, intra_encode(resid[..., None], scale, zigzag)


def histogram(sym, lo, nbins):
    """Per-symbol histogram over [lo, lo+nbins) with out-of-range values clamped into the
    end bins (the per-rank histogram the all-gather exchanges; stats_marg at
    ivclab/entropy/entropy.py:6-29 bins symbols the same way with pixel_range as edges)."""
    v = np.clip(np.asarray(sym, dtype=np.int64).ravel() - lo, 0, nbins - 1)
    return np.bincount(v, minlength=nbins).astype(np.int64)


# ---------------------------------------------------------------- zero-run coding -------
def zerorun_encode(flat, eob=4000, block_size=64):
    """ZeroRunCoder.encode (ivclab/entropy/zerorun.py:10-43): blocks in (h w c) order; per
    block the coefficients up to the last nonzero one (the scan starts at block_size - 1,
    :21-23), each nonzero value as itself and each zero run as (0, run length) (:29-37),
    then EOB (:38); an all-zero block is just EOB (:25-27).  int32 stream."""
    x = np.asarray(flat)
    rows = x.reshape(-1, x.shape[-1])
    out = []
    for blk in rows:
        last = block_size - 1
        while last >= 0 and blk[last] == 0:
            last -= 1
        if last == -1:
            out.append(eob)
            continue
        i = 0
        while i <= last:
            v = blk[i]
            if v == 0:
                run = 1
                while i + run <= last and blk[i + run] == 0:
                    run += 1
                out.extend([0, run])
                i += run
            else:
                out.append(int(v))
                i += 1
        out.append(eob)
    return np.array(out, dtype=np.int32)


def zerorun_encode_fast(flat, eob=4000, block_size=64):
    """Vectorised zerorun_encode for int32 blocks of exactly block_size coefficients (same
    stream; used for the larger parity cases)."""
    x = np.ascontiguousarray(flat, dtype=np.int32).reshape(-1, block_size)
    nz = x != 0
    any_nz = nz.any(1)
    last = np.where(any_nz, block_size - 1 - np.argmax(nz[:, ::-1], axis=1), -1)
    pos = np.arange(block_size)
    inside = pos[None, :] <= last[:, None]
    prev_nz = np.concatenate([np.ones((x.shape[0], 1), bool), nz[:, :-1]], axis=1)
    start = inside & ~nz & prev_nz                       # first zero of a run
    # symbols per element: nonzero -> 1, run start -> 2, other zeros inside -> 0
    per = np.where(inside & nz, 1, 0) + np.where(start, 2, 0)
    cnt = per.sum(1) + 1                                 # + EOB
    offs = np.concatenate([[0], np.cumsum(cnt)])
    out = np.empty(offs[-1], np.int32)
    within = np.cumsum(per, axis=1) - per                # exclusive position inside the block
    base = offs[:-1, None] + within
    r, c = np.nonzero(inside & nz)
    out[base[r, c]] = x[r, c]
    r, c = np.nonzero(start)
    out[base[r, c]] = 0
    # run length = distance to the next nonzero (which exists: the run ends before last)
    nxt = np.where(nz, pos[None, :], block_size)
    nxt = np.minimum.accumulate(nxt[:, ::-1], axis=1)[:, ::-1]
    out[base[r, c] + 1] = nxt[r, c] - c
    out[offs[1:] - 1] = eob
    return out


def zerorun_decode(encoded, original_shape, eob=4000, block_size=64):
    """ZeroRunCoder.decode (ivclab/entropy/zerorun.py:46-88), including its errors:
    ValueError on a stream that ends inside a block (:65-66), IndexError when it ends right
    after a 0 (the run length read at :74), ValueError when a block grows past block_size
    (:79-80) and when fewer blocks than h*w*c are found (:85-86); symbols after the last
    expected block are ignored (:62).  Returns [h, w, c, block_size] int32."""
    h, w, c = original_shape
    expected = h * w * c
    blocks = []
    i = 0
    n = len(encoded)
    while i < n and len(blocks) < expected:
        blk = []
        while True:
            if i >= n:
                raise ValueError("Unexpected end of encoded symbols")
            s = encoded[i]
            i += 1
            if s == eob:
                blk.extend([0] * (block_size - len(blk)))
                break
            elif s == 0:
                run = encoded[i]
                i += 1
                blk.extend([0] * run)
            else:
                blk.append(s)
            if len(blk) > block_size:
                raise ValueError(f"Block size exceeded: {len(blk)}")
        if len(blk) != block_size:
            raise ValueError(f"Incomplete block: {len(blk)}")
        blocks.append(blk)
    if len(blocks) != expected:
        raise ValueError(f"Expected {expected} blocks, got {len(blocks)}")
    return np.array(blocks, dtype=np.int32).reshape(h, w, c, block_size)


# ---------------------------------------------------------------- symbol statistics -----
def stats_marg(image, pixel_range):
    """stats_marg (ivclab/entropy/entropy.py:6-29): np.histogram of the float64-cast,
    flattened data over the bin edges pixel_range, divided by the number of samples.
    Pinned by tests/golden/stats.npz (the reference's own stats_marg, imported with the
    `ivclab` / `ivclab.entropy` package __init__ files bypassed: make_golden.py make_stats)."""
    flat = np.asarray(image).astype(np.float64).flatten()
    counts, _ = np.histogram(flat, bins=pixel_range)
    return counts / flat.size


def smooth_pmf(pmf, epsilon=1e-9):
    """entropy.py:31-35."""
    pmf = pmf + epsilon
    pmf /= pmf.sum()
    return pmf


def calc_entropy(pmf):
    """entropy.py:36-51."""
    nonzero_pmf = pmf[pmf > 0]
    return -np.sum(nonzero_pmf * np.log2(nonzero_pmf))


# ---------------------------------------------------------------- colour ----------------
YCC_M = np.array([[0.299, 0.587, 0.114], [-0.168736, -0.331264, 0.5],
                  [0.5, -0.418688, -0.081312]])


def rgb2ycbcr(image):
    """color.py:15-38 — the same NumPy matmul (OpenBLAS dgemm) and offset add."""
    return image @ YCC_M.T + np.array([0, 128, 128])


def rgb2ycbcr_fma(image):
    """The arithmetic the GPU kernel performs: per output channel
    fma(b, M[c,2], fma(g, M[c,1], r * M[c,0])) + offset, written with exact float64
    operations (an FMA is emulated as an error-free product + sum).  Equal to rgb2ycbcr on
    OpenBLAS's k-order FMA kernels (checked in tests/test_oracle_golden.py)."""
    x = np.asarray(image, dtype=np.float64)
    out = np.empty(x.shape, np.float64)
    from fractions import Fraction  # exact rational arithmetic: small inputs only
    flat_in = x.reshape(-1, 3)
    flat_out = out.reshape(-1, 3)
    off = (0.0, 128.0, 128.0)
    for i, (r, g, b) in enumerate(flat_in):
        for c in range(3):
            acc = float(Fraction(r) * Fraction(YCC_M[c, 0]))
            acc = float(Fraction(g) * Fraction(YCC_M[c, 1]) + Fraction(acc))
            acc = float(Fraction(b) * Fraction(YCC_M[c, 2]) + Fraction(acc))
            flat_out[i, c] = acc + off[c]
    return out


def ycbcr2rgb(image):
    """color.py:40-63."""
    Y = image[:, :, 0]
    Cb = image[:, :, 1] - 128.0
    Cr = image[:, :, 2] - 128.0
    R = Y + 1.402 * Cr
    G = Y - 0.344136 * Cb - 0.714136 * Cr
    B = Y + 1.772 * Cb
    return np.clip(np.stack([R, G, B], axis=-1), 0, 255)


def rgb2gray(image):
    """color.py:3-13."""
    return np.mean(image, axis=-1, keepdims=True)
