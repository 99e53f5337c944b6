"""ivclab.entropy (reference ivclab/entropy/__init__.py:1-4: entropy, probability,
huffman, zerorun).  The chapter-2 joint/conditional statistics of probability.py are
left out."""
from .entropy import calc_entropy, min_code_length, smooth_pmf, stats_marg
from .huffman import HuffmanCoder
from .zerorun import ZeroRunCoder
from . import entropy, huffman, zerorun  # noqa: F401
from .._scope import out_of_scope

__all__ = ["calc_entropy", "min_code_length", "smooth_pmf", "stats_marg", "HuffmanCoder",
           "ZeroRunCoder"]

__getattr__ = out_of_scope(__name__, {
    n: "ivclab/entropy/probability.py: chapter-2 histogram statistics and plots"
    for n in ("basic_histo", "count_rgb_histogram", "plot_histogram",
              "plot_image_and_joint_histogram", "stats_joint", "stats_cond")})
