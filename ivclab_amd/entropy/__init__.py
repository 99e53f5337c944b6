"""ivclab.entropy's block-codec part on the MI355X: the zero-run coder (the Huffman
coder needs the absent `constriction` wheel and stays out of scope)."""
from .stats import huffman_bounds, smooth_pmf, stats_marg_from_counts  # noqa: F401
from .zerorun import ZeroRunCoder  # noqa: F401
