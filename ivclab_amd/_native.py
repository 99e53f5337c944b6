"""ctypes binding of libivc.so (the C-ABI declared in include/ivc.h).

There is no CPU fallback: if the shared library is missing, was built for another
architecture, or no gfx950 device is visible, every hot-path call raises.  The library is
built in-tree by `python -m ivclab_amd.build` (or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as _ct
from ctypes import addressof as _addressof, c_char as _c_char
import math
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libivc.so")

# ivc_dtype codes (include/ivc.h)
DTYPE_CODE = {
    np.dtype(np.uint8): 1, np.dtype(np.int8): 2, np.dtype(np.uint16): 3,
    np.dtype(np.int16): 4, np.dtype(np.uint32): 5, np.dtype(np.int32): 6,
    np.dtype(np.uint64): 7, np.dtype(np.int64): 8, np.dtype(np.float32): 9,
    np.dtype(np.float64): 10,
}
F32, F64 = 9, 10
NORM_CODE = {None: 0, "backward": 0, "ortho": 1, "forward": 2}
ME_NUMPY, ME_EXACT_U8 = 0, 1

E_ARG, E_DTYPE, E_SHAPE, E_DEVICE, E_NOMEM = -1, -2, -3, -4, -5


class IvcError(RuntimeError):
    """Device-side failure reported by libivc (status IVC_E_DEVICE / IVC_E_NOMEM)."""


_P, _I, _L = _ct.c_void_p, _ct.c_int, _ct.c_int64
_SIGS = {
    "ivc_last_error": ([], _ct.c_char_p),
    "ivc_version": ([], _I),
    "ivc_me_mfma_enabled": ([], _I),
    "ivc_device_count": ([], _I),
    "ivc_set_device": ([_I], _I),
    "ivc_device_ok": ([], _I),
    "ivc_release_scratch": ([], _I),
    "ivc_host_alloc": ([_L], _P),
    "ivc_host_free": ([_P], _I),
    "ivc_set_store_pace": ([_ct.c_double], _I),
    "ivc_store_pace": ([], _ct.c_double),
    "ivc_store_pace_late": ([], _ct.c_double),
    "ivc_store_pace_stats": ([_I, _P, _I], _I),
    "ivc_store_pace_reset_stats": ([], _I),
    "ivc_store_pace_trace": ([_I, _P, _I], _I),
    "ivc_store_pace_settle": ([_ct.c_double], _I),
    "ivc_set_histogram_occupancy": ([_I], _I),
    "ivc_histogram_occupancy": ([], _I),
    "ivc_dct8x8": ([_P, _I, _L, _P, _I, _I, _I], _I),
    "ivc_dct8x8_dev": ([_P, _I, _L, _P, _I, _I, _I, _P], _I),
    "ivc_dct8x8_image": ([_P, _I, _L, _L, _L, _P, _I, _I, _I], _I),
    "ivc_set_host_pipeline": ([_L], _I),
    "ivc_host_pipeline": ([], _L),
    "ivc_set_tuning": ([_I, _I], _I),
    "ivc_tuning": ([_I], _I),
    "ivc_dct8x8_image_dev": ([_P, _I, _L, _L, _L, _P, _I, _I, _I, _P], _I),
    "ivc_quantize": ([_P, _I, _L, _I, _P, _I, _P], _I),
    "ivc_quantize_dev": ([_P, _I, _L, _I, _P, _I, _P, _P], _I),
    "ivc_dequantize": ([_P, _I, _L, _I, _P, _I, _P], _I),
    "ivc_dequantize_dev": ([_P, _I, _L, _I, _P, _I, _P, _P], _I),
    "ivc_zigzag": ([_P, _L, _L, _I, _I, _P], _I),
    "ivc_zigzag_dev": ([_P, _L, _L, _I, _I, _P, _P], _I),
    "ivc_intra_encode": ([_P, _I, _L, _L, _L, _I, _P, _I, _I, _P], _I),
    "ivc_intra_encode_dev": ([_P, _I, _L, _L, _L, _I, _P, _I, _I, _P, _P, _ct.c_int32,
                              _ct.c_int32, _P], _I),
    "ivc_intra_encode_luma_dev": ([_P, _L, _L, _L, _P, _I, _P, _P], _I),
    "ivc_intra_decode": ([_P, _L, _P, _I, _I, _P], _I),
    "ivc_intra_decode_dev": ([_P, _L, _P, _I, _I, _P, _P], _I),
    "ivc_intra_decode_image": ([_P, _L, _L, _L, _I, _P, _I, _I, _P], _I),
    "ivc_intra_decode_image_dev": ([_P, _L, _L, _L, _I, _P, _I, _I, _P, _P], _I),
    "ivc_symbols2image": ([_P, _L, _L, _L, _L, _I, _P, _ct.c_int32, _I, _P, _P], _I),
    "ivc_symbols2image_dev": ([_P, _L, _L, _L, _L, _I, _P, _ct.c_int32, _I, _P, _P, _P], _I),
    "ivc_motion_estimate": ([_P, _P, _I, _L, _L, _L, _I, _I, _P], _I),
    "ivc_motion_estimate_dev": ([_P, _P, _I, _L, _L, _L, _I, _I, _P, _P], _I),
    "ivc_motion_compensate": ([_P, _I, _L, _L, _L, _L, _P, _I, _P], _I),
    "ivc_motion_compensate_dev": ([_P, _I, _L, _L, _L, _L, _P, _I, _P, _P], _I),
    "ivc_inter_encode_dev": ([_P, _L, _L, _L, _I, _P, _I, _I, _P, _P, _P], _I),
    "ivc_inter_encode_hist_dev": ([_P, _L, _L, _L, _I, _P, _I, _I, _P, _P, _P, _I, _I, _P], _I),
    "ivc_histogram_i32": ([_P, _L, _ct.c_int32, _ct.c_int32, _P], _I),
    "ivc_histogram_i32_dev": ([_P, _L, _ct.c_int32, _ct.c_int32, _P, _P], _I),
    "ivc_histogram_i64": ([_P, _L, _L, _ct.c_int32, _P], _I),
    "ivc_histogram_f64_edges": ([_P, _L, _P, _ct.c_int32, _P], _I),
    "ivc_histogram_f64_edges_dev": ([_P, _L, _P, _ct.c_int32, _P, _P], _I),
    "ivc_huffman_lengths": ([_P, _ct.c_int32, _P], _I),
    "ivc_huffman_encode": ([_P, _L, _ct.c_int32, _P, _ct.c_int32, _P, _L, _P], _I),
    "ivc_huffman_decode": ([_P, _L, _L, _ct.c_int32, _P, _ct.c_int32, _P], _I),
    "ivc_rgb2ycbcr": ([_P, _ct.c_int, _L, _P], _I),
    "ivc_rgb2ycbcr_dev": ([_P, _ct.c_int, _L, _P, _P], _I),
    "ivc_ycbcr2rgb": ([_P, _ct.c_int, _L, _L, _P], _I),
    "ivc_ycbcr2rgb_dev": ([_P, _ct.c_int, _L, _L, _P, _P], _I),
    "ivc_rgb2gray": ([_P, _ct.c_int, _L, _L, _P], _I),
    "ivc_rgb2gray_dev": ([_P, _ct.c_int, _L, _L, _P, _P], _I),
    "ivc_intra_symbols": ([_P, _ct.c_int, _L, _L, _L, _ct.c_int, _P, _ct.c_int32, _P, _L, _P], _I),
    "ivc_intra_symbols_dev": ([_P, _ct.c_int, _L, _L, _L, _ct.c_int, _P, _ct.c_int32, _P, _L, _P, _P], _I),
    "ivc_intra_symbols_hist_dev": ([_P, _ct.c_int, _L, _L, _L, _ct.c_int, _P, _ct.c_int32, _P, _L, _P,
                                    _P, _ct.c_int32, _ct.c_int32, _P], _I),
    "ivc_minmax_i32": ([_P, _L, _P], _I),
    "ivc_minmax_i32_dev": ([_P, _L, _P, _P], _I),
    "ivc_zerorun_encode": ([_P, _L, _ct.c_int32, _ct.c_int32, _ct.c_int32, _P, _L, _P], _I),
    "ivc_zerorun_encode_dev": ([_P, _L, _ct.c_int32, _ct.c_int32, _ct.c_int32, _P, _P, _L, _P], _I),
    "ivc_zerorun_decode": ([_P, _L, _L, _ct.c_int32, _ct.c_int32, _P, _P], _I),
    "ivc_zerorun_decode_dev": ([_P, _L, _L, _ct.c_int32, _ct.c_int32, _P, _P, _P], _I),
    "ivc_histogram_i64_dev": ([_P, _L, _L, _ct.c_int32, _P, _P], _I),
}
EXPORTS = tuple(_SIGS)

_lib = None
_lock = threading.Lock()
_device_checked = False


def _share_torch_hip_runtime() -> None:
    """Bind libivc to the HIP runtime torch ships, when torch is installed.

    torch-ROCm bundles its own libamdhip64 / libhsa-runtime64 (same SONAMEs as /opt/rocm's).
    Two HIP runtimes in one process cannot both own the GPU: whichever initialises second
    sees no device.  Loading torch's copies first (RTLD_GLOBAL) makes libivc's DT_NEEDED
    entries resolve to them by SONAME, so the process has exactly one runtime whatever the
    import order.  IVC_HIP_RUNTIME=system keeps /opt/rocm's runtime instead.
    """
    if os.environ.get("IVC_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    tlib = os.path.join(os.path.dirname(spec.origin), "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(tlib, name)
        if os.path.exists(p):
            _ct.CDLL(p, mode=_ct.RTLD_GLOBAL)


def load_library(path: str = LIB_PATH):
    """Load libivc.so and declare its signatures (no device is touched)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise ImportError(
                    f"ivclab_amd: native library {path} is missing; build it with "
                    "`python -m ivclab_amd.build` (hipcc --offload-arch=gfx950)")
            _share_torch_hip_runtime()
            lib = _ct.CDLL(path)
            for name, (args, res) in _SIGS.items():
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = res
            _lib = lib
    return _lib


def lib():
    """The loaded library, after checking once that a gfx950 device is present."""
    global _device_checked
    L = load_library()
    if not _device_checked:
        if L.ivc_device_count() < 1:
            raise IvcError("ivclab_amd: no HIP device visible; the block-codec path runs only "
                           "on an MI355X (gfx950) — there is no CPU fallback")
        if not L.ivc_device_ok():
            raise IvcError("ivclab_amd: current HIP device is not gfx950 (MI355X)")
        _device_checked = True
    return L


_fast = False          # False: not tried yet; None: unavailable


def fast():
    """The per-block call accelerator (ivc_pyfast.c: the small-array fast paths of
    DiscreteCosineTransform and PatchQuant in one C step), bound to this process's libivc
    entry points after the device check; None when its module is missing (the ctypes path then
    serves those calls)."""
    global _fast
    if _fast is False:
        L = lib()
        try:
            import importlib.machinery
            import importlib.util
            import sysconfig
            path = os.path.join(_HERE, "_lib", "_ivcfast" + sysconfig.get_config_var("EXT_SUFFIX"))
            loader = importlib.machinery.ExtensionFileLoader("ivclab_amd._ivcfast", path)
            spec = importlib.util.spec_from_file_location("ivclab_amd._ivcfast", path, loader=loader)
            mod = importlib.util.module_from_spec(spec)
            loader.exec_module(mod)
            addr = lambda f: _ct.cast(f, _ct.c_void_p).value  # noqa: E731
            mod.set_entry_points(addr(L.ivc_dct8x8), addr(L.ivc_quantize), addr(L.ivc_dequantize))
            _fast = mod
        except (ImportError, OSError):
            _fast = None
    return _fast


def check(status: int, what: str = "ivc") -> None:
    """Map a libivc status to the exception class NumPy would raise for the same misuse."""
    if status == 0:
        return
    msg = (load_library().ivc_last_error() or b"").decode(errors="replace")
    if status in (E_SHAPE, E_DTYPE, E_ARG):
        raise ValueError(f"{what}: {msg}")
    if status == E_NOMEM:
        raise MemoryError(f"{what}: {msg}")
    raise IvcError(f"{what}: {msg}")


def ptr(a: np.ndarray) -> int:
    # Address of the first element.  a.ctypes.data builds a ctypes object per call (~1 us on the
    # GPU box's host, as long as the DCT kernel's host side of a per-block loop call): the
    # buffer address of a writable C-contiguous array is 3x cheaper; anything else (read-only,
    # strided, empty) takes the array interface.
    try:
        return _addressof(_c_char.from_buffer(a))
    except (TypeError, ValueError, BufferError):
        return a.__array_interface__["data"][0]


def pace_stats(encoder: int = 0):
    """Store-pacing measurements of the current device since the last reset
    (ivc_store_pace_stats), as a dict; None when no launch was measured."""
    out = np.zeros(10, np.float64)
    n = lib().ivc_store_pace_stats(encoder, out.ctypes.data, 10)
    check(min(n, 0), "pace_stats")
    if out[0] < 1:
        return None
    return {"launches_measured": int(out[0]), "launches_over_late_threshold": int(out[1]),
            "late_fraction_mean": round(float(out[2]), 4), "late_fraction_max": round(float(out[3]), 4),
            "rate_GBs": round(float(out[4]), 1), "late_fraction_last": round(float(out[5]), 4),
            "achieved_GBs_mean": round(float(out[6]), 1),
            "late_but_on_pace": int(out[8]), "lowest_failed_rate_GBs": round(float(out[9]), 1)}


def pace_trace(encoder: int = 0, max_records: int = 256):
    """Per-launch store-pacing trace since the last reset (ivc_store_pace_trace), oldest
    first: [rate GB/s, late fraction past the start-up, achieved GB/s, start lag us, first late
    slot past the start-up, next rate, late fraction of the start-up slots]."""
    out = np.zeros((max_records, 7), np.float64)
    n = lib().ivc_store_pace_trace(encoder, out.ctypes.data, max_records)
    check(min(n, 0), "pace_trace")
    return [[round(float(v), 4 if i in (1, 4, 6) else 1) for i, v in enumerate(r)] for r in out[:n]]


_PINNED_MIN = 1 << 20


def empty(shape, dtype) -> np.ndarray:
    """np.empty in a page-locked block of the library's host pool (ivc_host_alloc) when the
    array is large (>= 1 MiB): the device writes it with one DMA and no staging copy.  The
    block returns to the pool when the array (and every view of it) is garbage collected.
    Falls back to np.empty when no device library is usable or pinning fails."""
    dtype = np.dtype(dtype)
    shape = tuple(int(d) for d in (shape if np.iterable(shape) else (shape,)))
    count = math.prod(shape)                 # (np.prod costs ~5 us per call: per-block loops)
    nbytes = count * dtype.itemsize
    if nbytes < _PINNED_MIN:
        return np.empty(shape, dtype)
    try:
        L = lib()
    except (ImportError, IvcError):
        return np.empty(shape, dtype)
    p = L.ivc_host_alloc(nbytes)
    if not p:
        return np.empty(shape, dtype)
    buf = (_ct.c_char * nbytes).from_address(p)
    fin = weakref.finalize(buf, L.ivc_host_free, p)
    fin.atexit = False
    return np.frombuffer(buf, dtype=dtype, count=count).reshape(shape)


def empty_like(a) -> np.ndarray:
    a = np.asarray(a)
    return empty(a.shape, a.dtype)


# ivc_set_tuning keys (include/ivc.h enum ivc_tuning_key)
TUNE = {"zr_chunks": 0, "sym_chunks": 1, "s2i_chunks": 2, "inter_chunks": 3, "s2i_no_fallback": 4,
        "f64_me": 5, "tiny_server": 6}


def set_tuning(name: str, value: int) -> int:
    """Set one pipeline tuning override (0 restores the library's choice); returns the previous
    value."""
    L = lib()
    key = TUNE[name]
    prev = int(L.ivc_tuning(key))
    check(L.ivc_set_tuning(key, int(value)), "ivc_set_tuning")
    return prev


def table_arg(table: np.ndarray) -> np.ndarray:
    """3x8x8 table as 192 float64 values (exact for float32/float64 tables)."""
    t = np.ascontiguousarray(table, dtype=np.float64).reshape(-1)
    if t.size != 192:
        raise ValueError("quantization table must hold 3 x 8 x 8 values")
    return t
