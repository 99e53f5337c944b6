"""ivclab.signal.color (reference ivclab/signal/color.py:3-63): gfx950 colour kernels."""
from ivclab_amd.signal.color import rgb2gray, rgb2ycbcr, ycbcr2rgb

__all__ = ["rgb2gray", "rgb2ycbcr", "ycbcr2rgb"]
