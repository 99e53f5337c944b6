"""ivclab.entropy.entropy (reference ivclab/entropy/entropy.py:6-72)."""
from ivclab_amd.entropy.stats import calc_entropy, min_code_length, smooth_pmf, stats_marg

__all__ = ["stats_marg", "smooth_pmf", "calc_entropy", "min_code_length"]
