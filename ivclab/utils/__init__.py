"""ivclab.utils (reference ivclab/utils/__init__.py:1-3: io, metrics, shape)."""
from .io import imread, imshow
from .metrics import calc_mse, calc_psnr
from .shape import Patcher, ZigZag
from . import io, metrics, shape  # noqa: F401

__all__ = ["imread", "imshow", "calc_mse", "calc_psnr", "Patcher", "ZigZag"]
