"""ivclab.image's transform codec on the MI355X (IntraCodec).  The chapter-2 predictive and
YUV 4:2:0 codecs are outside the block-codec hot path."""
from .intracodec import IntraCodec  # noqa: F401
