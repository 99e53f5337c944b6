"""calc_mse / calc_psnr with the reference's formulas (ivclab/utils/metrics.py:3-39).
Not on the hot path; present so tests written against the reference's ch3 API (which
score a reconstruction with these) run unchanged."""
import numpy as np


def calc_mse(orig: np.ndarray, rec: np.ndarray):
    if orig.ndim == 2 and rec.ndim == 3:
        orig = np.stack([orig] * 3, axis=-1)
    elif orig.ndim == 3 and rec.ndim == 2:
        rec = np.stack([rec] * 3, axis=-1)
    assert orig.shape == rec.shape, f"Image shapes don't match after processing: {orig.shape} vs {rec.shape}"
    return np.mean((orig.astype(np.float64) - rec.astype(np.float64)) ** 2)


def calc_psnr(orig: np.ndarray, rec: np.ndarray, maxval=255):
    return 20 * np.log10(maxval / np.sqrt(calc_mse(orig, rec)))
