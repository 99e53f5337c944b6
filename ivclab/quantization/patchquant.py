"""ivclab.quantization.patchquant (reference ivclab/quantization/patchquant.py:3-78)."""
from ivclab_amd.quantization.patchquant import PatchQuant

__all__ = ["PatchQuant"]
