"""ivclab.entropy's block-codec part on the MI355X: the zero-run coder (GPU), the symbol
statistics (GPU histogram + host pmf finish) and the host-side Huffman coder (libivc; the
reference's `constriction`-based trees are unavailable, so bitstreams are not pinned)."""
from .huffman import HuffmanCoder  # noqa: F401
from .stats import (calc_entropy, huffman_bounds, min_code_length, smooth_pmf,  # noqa: F401
                    stats_marg, stats_marg_from_counts)
from .zerorun import ZeroRunCoder  # noqa: F401
