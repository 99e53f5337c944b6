"""ivclab.signal hot-path subset: DiscreteCosineTransform (zigzag_scan lives in
ivclab_amd.signal.zigzag, as ivclab/signal/__init__.py:1-3 does not export it either)."""
from .dct import DiscreteCosineTransform  # noqa: F401
