"""ivclab.quantization (reference ivclab/quantization/__init__.py:2)."""
from .patchquant import PatchQuant
from . import patchquant  # noqa: F401

__all__ = ["PatchQuant"]
