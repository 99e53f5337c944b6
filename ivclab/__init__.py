"""`ivclab` — the reference's package name, backed by the MI355X block-codec core.

The reference's callers (tests/ch3.py, exercises/ch3, exercises/ch4) import
`ivclab.signal`, `ivclab.quantization`, `ivclab.utils`, `ivclab.video`,
`ivclab.entropy` and `ivclab.image` directly.  This package gives those module
paths and names, each one the `ivclab_amd` object that runs on the gfx950 kernels
(libivc.so), so the callers run unchanged with only this repository on
`PYTHONPATH`: no prelude, and no `constriction` wheel (the reference's
`ivclab/__init__.py` pulls it in through `entropy/huffman.py:2`).

Like the reference's `ivclab/__init__.py:1-5`, the root star-imports entropy, image,
quantization, utils and video, and not signal.  Names that live outside the
block-codec hot path (chapter-1/2 filters, predictive and 4:2:0 codecs, joint
statistics, `IntraCodecAdaptive`) are not provided: importing one raises ImportError
naming the reason.
"""
from .entropy import *  # noqa: F401,F403
from .image import *  # noqa: F401,F403
from .quantization import *  # noqa: F401,F403
from .utils import *  # noqa: F401,F403
from .video import *  # noqa: F401,F403
from . import entropy, image, quantization, signal, utils, video  # noqa: F401
