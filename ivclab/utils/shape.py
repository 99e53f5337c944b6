"""ivclab.utils.shape (reference ivclab/utils/shape.py:4-65): ZigZag and Patcher."""
from ivclab_amd.utils.shape import Patcher, ZigZag

__all__ = ["ZigZag", "Patcher"]
