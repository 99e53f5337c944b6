"""ivclab.video (reference ivclab/video/__init__.py:1-2)."""
from .motion import MotionCompensator
from .videocodec import VideoCodec
from . import motion, videocodec  # noqa: F401

__all__ = ["MotionCompensator", "VideoCodec"]
