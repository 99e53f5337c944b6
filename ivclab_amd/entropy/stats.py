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
