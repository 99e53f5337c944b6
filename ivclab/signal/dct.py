"""ivclab.signal.dct (reference ivclab/signal/dct.py:4-46): the gfx950 8x8 DCT/IDCT."""
from ivclab_amd.signal.dct import DiscreteCosineTransform

__all__ = ["DiscreteCosineTransform"]
