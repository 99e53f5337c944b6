"""ivclab.utils.io (reference ivclab/utils/io.py:5-23)."""
from ivclab_amd.utils.io import imread, imshow

__all__ = ["imread", "imshow"]
