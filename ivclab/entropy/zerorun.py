"""ivclab.entropy.zerorun (reference ivclab/entropy/zerorun.py:4-88): gfx950 zero-run coder."""
from ivclab_amd.entropy.zerorun import ZeroRunCoder

__all__ = ["ZeroRunCoder"]
