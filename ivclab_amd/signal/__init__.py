"""ivclab.signal hot-path subset: DiscreteCosineTransform and the colour conversions
(zigzag_scan lives in ivclab_amd.signal.zigzag, as ivclab/signal/__init__.py does not export
it either)."""
from .color import rgb2gray, rgb2ycbcr, ycbcr2rgb  # noqa: F401
from .dct import DiscreteCosineTransform  # noqa: F401
