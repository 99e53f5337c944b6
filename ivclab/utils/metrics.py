"""ivclab.utils.metrics (reference ivclab/utils/metrics.py:3-39)."""
from ivclab_amd.utils.metrics import calc_mse, calc_psnr

__all__ = ["calc_mse", "calc_psnr"]
