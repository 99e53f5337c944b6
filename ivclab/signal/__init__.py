"""ivclab.signal (reference ivclab/signal/__init__.py:1-3: signal, color, dct).

`zigzag_scan` is reached as `ivclab.signal.zigzag.zigzag_scan`, as in the reference."""
from .color import rgb2gray, rgb2ycbcr, ycbcr2rgb
from .dct import DiscreteCosineTransform
from . import color, dct, zigzag  # noqa: F401
from .._scope import out_of_scope

__all__ = ["rgb2gray", "rgb2ycbcr", "ycbcr2rgb", "DiscreteCosineTransform"]

__getattr__ = out_of_scope(__name__, {
    n: "ivclab/signal/signal.py: chapter-1 resampling and filtering"
    for n in ("downsample", "upsample", "interpolation_upsample", "lowpass_filter",
              "FilterPipeline", "filter_img")})
