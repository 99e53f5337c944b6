from .motion import MotionCompensator  # noqa: F401
from .videocodec import VideoCodec  # noqa: F401
