"""ivclab.video.motion (reference ivclab/video/motion.py:3-97): gfx950 ME/MC."""
from ivclab_amd.video.motion import MotionCompensator

__all__ = ["MotionCompensator"]
