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

`install_as_ivclab()` registers these modules under the reference's import paths
(ivclab.signal, ivclab.signal.dct, ...) so unchanged callers pick them up.
"""
import importlib
import sys
import types

from .quantization import PatchQuant  # noqa: F401
from .signal import DiscreteCosineTransform  # noqa: F401
from .utils import Patcher, ZigZag  # noqa: F401
from .entropy import HuffmanCoder, ZeroRunCoder  # noqa: F401
from .image import IntraCodec  # noqa: F401
from .video import MotionCompensator, VideoCodec  # noqa: F401

__version__ = "0.1.0"

_ALIASES = {
    "ivclab.signal": "ivclab_amd.signal",
    "ivclab.signal.dct": "ivclab_amd.signal.dct",
    "ivclab.signal.zigzag": "ivclab_amd.signal.zigzag",
    "ivclab.signal.color": "ivclab_amd.signal.color",
    "ivclab.quantization": "ivclab_amd.quantization",
    "ivclab.quantization.patchquant": "ivclab_amd.quantization.patchquant",
    "ivclab.utils": "ivclab_amd.utils",
    "ivclab.utils.shape": "ivclab_amd.utils.shape",
    "ivclab.utils.metrics": "ivclab_amd.utils.metrics",
    "ivclab.utils.io": "ivclab_amd.utils.io",
    "ivclab.video": "ivclab_amd.video",
    "ivclab.video.motion": "ivclab_amd.video.motion",
    "ivclab.video.videocodec": "ivclab_amd.video.videocodec",
    "ivclab.entropy": "ivclab_amd.entropy",
    "ivclab.entropy.huffman": "ivclab_amd.entropy.huffman",
    "ivclab.image": "ivclab_amd.image",
    "ivclab.image.intracodec": "ivclab_amd.image.intracodec",
    "ivclab.entropy.zerorun": "ivclab_amd.entropy.zerorun",
}


def install_as_ivclab() -> None:
    """Make `import ivclab.<hot-path module>` resolve to this package's modules."""
    root = sys.modules.get("ivclab")
    if root is None:
        root = types.ModuleType("ivclab")
        root.__path__ = []  # namespace-like: only the aliased submodules resolve
        sys.modules["ivclab"] = root
    for name, target in _ALIASES.items():
        mod = importlib.import_module(target)
        sys.modules[name] = mod
        parent, _, leaf = name.rpartition(".")
        setattr(sys.modules[parent], leaf, mod)
    for cls in (PatchQuant, DiscreteCosineTransform, Patcher, ZigZag, MotionCompensator,
                ZeroRunCoder, HuffmanCoder, IntraCodec, VideoCodec):
        setattr(root, cls.__name__, cls)
