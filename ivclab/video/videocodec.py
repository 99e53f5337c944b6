"""ivclab.video.videocodec (reference ivclab/video/videocodec.py:12-86)."""
from ivclab_amd.video.videocodec import VideoCodec

__all__ = ["VideoCodec"]
