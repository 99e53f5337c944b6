from .motion import MotionCompensator  # noqa: F401
