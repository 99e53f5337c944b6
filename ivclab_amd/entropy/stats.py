"""Host-side finish of the global symbol statistics: the probability mass function the
reference's Huffman training builds (ivclab/entropy/entropy.py:6-35, intracodec.py:
161-166) from histogram counts that the GPU computed (ivc_histogram_i32) and the ranks
all-gathered.  Tiny arrays (one entry per alphabet symbol): NumPy, same operations as the
reference so the table is bit-identical."""
from __future__ import annotations

import numpy as np


def huffman_bounds(sym_min: int, sym_max: int, safety_margin: int = 20):
    """IntraCodec.train_huffman_from_image's alphabet (intracodec.py:161-163)."""
    return int(sym_min) - safety_margin, int(sym_max) + safety_margin + 1


def bounds_from_histogram(hist, lo):
    """(min, max) of the symbols a guarded histogram counted — hist[0] = values below lo,
    hist[1 + k] = value lo + k, hist[-1] = values past the range — or None when any symbol
    fell outside the range (the caller then takes the exact min/max path)."""
    h = np.asarray(hist)
    if h[0] or h[-1]:
        return None
    nz = np.flatnonzero(h[1:-1])
    if nz.size == 0:
        return None
    return lo + int(nz[0]), lo + int(nz[-1])


def counts_over(hist, lo, b0, b1):
    """np.histogram counts of the guarded histogram's symbols over the unit edges
    arange(b0, b1) (last bin closed), given that every symbol lies in [lo, lo + nbins)."""
    h = np.asarray(hist)[1:-1]
    v = np.arange(b0, b1 - 1)
    k = v - lo
    out = np.where((k >= 0) & (k < h.size), h[np.clip(k, 0, h.size - 1)], 0).astype(np.int64)
    last = b1 - 1 - lo                          # the closed last bin also holds value b1 - 1
    if out.size and 0 <= last < h.size:
        out[-1] += h[last]
    return out


def stats_marg_from_counts(counts, total=None):
    """stats_marg (entropy.py:6-29) given np.histogram's counts: counts / number of
    samples (float64)."""
    counts = np.asarray(counts)
    n = counts.sum() if total is None else total
    return counts / n


def smooth_pmf(pmf, epsilon=1e-9):
    """entropy.py:31-35."""
    pmf = pmf + epsilon
    pmf /= pmf.sum()
    return pmf


def entropy_bits(pmf):
    """Shannon entropy in bits per symbol of a (smoothed) pmf."""
    p = np.asarray(pmf, dtype=np.float64)
    p = p[p > 0]
    return float(-(p * np.log2(p)).sum())


def stats_marg(image, pixel_range):
    """entropy.py:6-29 — np.histogram(image.astype(float64).flatten(), bins=pixel_range)
    / image.size, counted on the GPU.

    Integer images over unit-spaced integer edges (the symbol and pixel statistics of the
    codec, including the int64 symbol / motion-vector arrays of the chapter-4 exercises) take
    the integer histogram kernels on the raw values: np.histogram drops values
    outside [edges[0], edges[-1]] and closes the last bin; the kernel clamps, so two guard
    bins on each side absorb the out-of-range values and the top edge value is folded into
    the last bin.  Everything else — float images, any edges, an int bin count or a binning
    rule — takes the edge kernel on the float64-cast values over the edges np.histogram
    itself would use (np.histogram_bin_edges: same validation, same errors), with
    np.histogram's comparisons: edges[i] <= x < edges[i+1], last bin closed, NaN and
    out-of-range values dropped."""
    from .. import _native as N
    a = np.asarray(image)
    edges = np.asarray(pixel_range)
    unit_int = (edges.ndim == 1 and edges.size >= 2 and np.issubdtype(edges.dtype, np.integer)
                and bool(np.all(np.diff(edges) == 1)))
    # Integer data over unit-spaced integer edges inside (-2^53, 2^53): every value lands in the
    # same bin before and after the reference's float64 cast (values within the edges are exact
    # in float64; a value beyond +-2^53 casts to something beyond the edges either way), so the
    # raw values are counted by the integer kernels (int32 when values and bins fit, else int64)
    int_data = np.issubdtype(a.dtype, np.integer) or a.dtype == np.bool_
    if unit_int and int_data and -2**53 < int(edges[0]) and int(edges[-1]) < 2**53 \
            and edges.size - 1 + 3 <= np.iinfo(np.int32).max:
        lo, nb = int(edges[0]), edges.size - 1
        x = np.ascontiguousarray(a.ravel())
        hist = np.zeros(nb + 3, np.int64)              # [< lo | lo .. lo+nb-1 | lo+nb | > lo+nb]
        i32 = np.iinfo(np.int32)
        fits32 = (x.dtype == np.bool_ or (x.dtype.itemsize <= 4 and x.dtype != np.uint32)) \
            and i32.min <= lo - 1 and lo + nb + 1 <= i32.max
        if fits32:
            x32 = x.astype(np.int32, copy=False)
            N.check(N.lib().ivc_histogram_i32(N.ptr(x32), x32.size, lo - 1, nb + 3, N.ptr(hist)),
                    "stats_marg")
        else:
            if x.dtype == np.uint64 and x.size and x.max() > np.iinfo(np.int64).max:
                x = np.minimum(x, np.uint64(np.iinfo(np.int64).max))   # all beyond the edges
            x64 = x.astype(np.int64, copy=False)
            N.check(N.lib().ivc_histogram_i64(N.ptr(x64), x64.size, lo - 1, nb + 3, N.ptr(hist)),
                    "stats_marg")
        counts = hist[1:nb + 1].copy()
        counts[-1] += hist[nb + 1]
        return counts / x.size
    flat = np.ascontiguousarray(a.astype(np.float64).flatten())
    bin_edges = np.ascontiguousarray(np.histogram_bin_edges(flat, bins=pixel_range), np.float64)
    if bin_edges.size - 1 > np.iinfo(np.int32).max:
        raise ValueError("stats_marg: too many bins")
    counts = np.zeros(bin_edges.size - 1, np.int64)
    if flat.size and counts.size:
        N.check(N.lib().ivc_histogram_f64_edges(N.ptr(flat), flat.size, N.ptr(bin_edges),
                                                bin_edges.size, N.ptr(counts)), "stats_marg")
    return counts / flat.size


def calc_entropy(pmf, eps=1e-8):
    """entropy.py:36-51."""
    nonzero_pmf = pmf[pmf > 0]
    return -np.sum(nonzero_pmf * np.log2(nonzero_pmf))


def min_code_length(target_pmf, common_pmf, eps=1e-8):
    """entropy.py:53-71."""
    common_pmf = common_pmf + eps
    return -np.sum(target_pmf * np.log2(common_pmf))
