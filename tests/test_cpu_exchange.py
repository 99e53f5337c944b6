"""The one-pass Huffman-table exchange (bench.py leg_symbols, ivclab_amd/entropy/stats.py):
a histogram over a fixed symbol range with a guard bin at each end yields the alphabet bounds
IntraCodec.train_huffman_from_image takes (min - 20, max + 21: intracodec.py:161-166) and the
np.histogram counts over arange(bounds) that stats_marg computes (entropy.py:6-29), or
declines when a symbol lies outside the range.  Host arithmetic only (no GPU)."""
import numpy as np
import pytest

from ivclab_amd.entropy.stats import bounds_from_histogram, counts_over, huffman_bounds
from oracle import ivc_oracle as O

LO, NB = -4096, 8192


def guarded(sym):
    return O.histogram(sym, LO - 1, NB + 2)


@pytest.mark.parametrize("seed", range(6))
def test_bounds_and_counts_match_two_pass(seed):
    rng = np.random.default_rng(seed)
    sym = rng.integers(-60, 60, 50_000).astype(np.int32)
    sym[::97] = 4000                                            # EOB
    if seed % 2:
        sym[5] = LO                                             # range ends
        sym[6] = LO + NB - 1
    h = guarded(sym)
    mn, mx = bounds_from_histogram(h, LO)
    assert (mn, mx) == (int(sym.min()), int(sym.max()))
    b0, b1 = huffman_bounds(mn, mx)
    want, _ = np.histogram(sym.astype(np.float64), bins=np.arange(b0, b1))
    assert np.array_equal(counts_over(h, LO, b0, b1), want)


def test_outside_the_range_declines():
    for bad in (LO - 1, LO + NB, 1 << 30, -(1 << 30)):
        sym = np.array([0, 1, bad, 4000], np.int32)
        assert bounds_from_histogram(guarded(sym), LO) is None
    assert bounds_from_histogram(np.zeros(NB + 2, np.int64), LO) is None
