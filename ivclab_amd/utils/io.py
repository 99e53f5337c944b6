"""Image I/O of the drop-in `ivclab.utils` (ivclab/utils/io.py:5-23).

Not on the hot path: the reference's callers load their test images with `imread` before
handing them to the block codec (tests/ch3.py:3,13; exercises/ch3, ch4), so `from
ivclab.utils import imread` has to resolve under `install_as_ivclab()`.  Same behaviour:
PIL opens the file and NumPy takes the decoded pixels as they are (no dtype or channel
conversion); `imshow` draws on a matplotlib axis (imported only when called).
"""
import numpy as np


def imread(filepath: str):
    """io.py:5-8: np.asarray of the PIL image (uint8 [H, W, C] for RGB, [H, W] for L)."""
    from PIL import Image
    with Image.open(filepath) as data:
        img = np.asarray(data)
    return img


def imshow(ax, img: np.ndarray, title=None, hide_ticks=True):
    """io.py:10-23: grey colour map for a single-channel image, no ticks by default."""
    if img.shape[-1] == 1:
        ax.imshow(img, cmap="gray")
    else:
        ax.imshow(img)
    if title is not None:
        ax.set_title(title)
    if hide_ticks:
        ax.set_xticks([])
        ax.set_yticks([])
