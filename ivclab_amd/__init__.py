"""ivclab_amd — MI355X-native block-codec core of the TUM IVC lab codebase (n2oblife/ivclab).

Hot path: 8x8 DCT/IDCT (ivclab.signal), JPEG-table quantisation + zig-zag
(ivclab.quantization, ivclab.utils.shape), full-search block-matching ME/MC
(ivclab.video.motion), behind the reference's own class API.  Arithmetic runs in
hand-written gfx950 kernels (libivc.so, C-ABI in include/ivc.h) and reproduces the
reference's NumPy/SciPy results bit for bit; there is no CPU fallback.

    from ivclab_amd.signal import DiscreteCosineTransform
    from ivclab_amd.quantization import PatchQuant
    from ivclab_amd.utils import ZigZag, Patcher
    from ivclab_amd.signal.zigzag import zigzag_scan
    from ivclab_amd.video import MotionCompensator, VideoCodec
    from ivclab_amd.entropy import ZeroRunCoder

The repository also ships the top-level `ivclab` package (ivclab/), which exposes these
objects under the reference's import paths (ivclab.signal, ivclab.signal.dct, ...), so the
reference's callers run unchanged with the repository on PYTHONPATH.
"""
import importlib
import os
import sys

from .quantization import PatchQuant  # noqa: F401
from .signal import DiscreteCosineTransform  # noqa: F401
from .utils import Patcher, ZigZag  # noqa: F401
from .entropy import HuffmanCoder, ZeroRunCoder  # noqa: F401
from .image import IntraCodec  # noqa: F401
from .video import MotionCompensator, VideoCodec  # noqa: F401

__version__ = "0.1.0"

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def install_as_ivclab():
    """Import and return the repository's own `ivclab` package (ivclab/ next to this one).

    Callers no longer need this: with the repository on `PYTHONPATH`, `import ivclab...`
    resolves to that package directly.  It stays for code written against earlier rounds;
    it puts the repository root on `sys.path` when it is missing, and refuses to proceed
    when a different `ivclab` (e.g. the reference's) is already imported."""
    mod = sys.modules.get("ivclab")
    if mod is None:
        if _ROOT not in sys.path:
            sys.path.insert(0, _ROOT)
        mod = importlib.import_module("ivclab")
    where = os.path.dirname(os.path.abspath(getattr(mod, "__file__", "") or ""))
    if os.path.dirname(where) != _ROOT:
        raise ImportError(f"another 'ivclab' package is already imported from {where}")
    return mod
