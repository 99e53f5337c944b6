"""ivclab.image (reference ivclab/image/__init__.py:1-3).  Only the transform codec is on
the block-codec hot path; the chapter-2 predictive and 4:2:0 codecs and
IntraCodecAdaptive are left out."""
from .intracodec import IntraCodec
from . import intracodec  # noqa: F401
from .._scope import out_of_scope

__all__ = ["IntraCodec"]

__getattr__ = out_of_scope(__name__, {
    "IntraCodecAdaptive": "ivclab/image/intracodec.py:244-306: pickles an attribute the "
                          "reference HuffmanCoder does not have",
    "single_pixel_predictor": "ivclab/image/predictive.py: chapter-2 predictive coding",
    "three_pixels_predictor": "ivclab/image/predictive.py: chapter-2 predictive coding",
    "yuv420compression": "ivclab/image/yuv420codec.py: chapter-1 4:2:0 codec",
    "pad_image": "ivclab/image/yuv420codec.py: chapter-1 4:2:0 codec",
    "crop_image": "ivclab/image/yuv420codec.py: chapter-1 4:2:0 codec"})
