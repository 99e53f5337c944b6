"""ivclab.image.intracodec (reference ivclab/image/intracodec.py:11-241)."""
from ivclab_amd.image.intracodec import IntraCodec

__all__ = ["IntraCodec"]
