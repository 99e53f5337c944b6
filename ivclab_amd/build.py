"""Build libivc.so in-tree for gfx950:  python -m ivclab_amd.build [-v]

hipcc compiles the HIP translation units (SOURCES) into ivclab_amd/_lib/libivc.so.  Flags that
matter for parity: -ffp-contract=off (no fused multiply-add: pocketfft / NumPy round every
product and sum separately) and no fast-math.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_lib", "libivc.so")
SOURCES = ["ivc_kernels.hip", "ivc_motion.hip", "ivc_me_mfma.hip", "ivc_me_f64.hip", "ivc_entropy.hip",
           "ivc_decode.hip", "ivc_color.hip", "ivc_huffman.hip", "ivc_capi.hip"]
# per-file code-generation flags (ivc_me_f64.hip's header says why)
FILE_FLAGS = {"ivc_me_f64.hip": ["-fno-slp-vectorize"]}
HEADERS = ["ivc_math.h", "ivc_internal.h", os.path.join("..", "..", "include", "ivc.h")]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libivc.so)")


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [__file__]
    return all(os.path.getmtime(d) <= t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)


PYFAST_SRC = os.path.join(CSRC, "ivc_pyfast.c")


def pyfast_path() -> str:
    import sysconfig
    return os.path.join(HERE, "_lib", "_ivcfast" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_pyfast(verbose: bool = False) -> str:
    """The CPython/NumPy accelerator of the per-block calls (ivc_pyfast.c): gcc, host only."""
    import sysconfig
    import numpy as np
    out = pyfast_path()
    if os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(PYFAST_SRC),
                                                            os.path.getmtime(__file__)):
        return out
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        raise RuntimeError("gcc not found (needed for the per-block call accelerator)")
    tmp = out + ".tmp"
    cmd = [cc, "-O2", "-shared", "-fPIC", "-Wall", "-I" + sysconfig.get_paths()["include"],
           "-I" + np.get_include(), "-o", tmp, PYFAST_SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gcc failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile each translation unit to an object (in parallel, under ivclab_amd/_lib/obj),
    then link the shared library.  The per-block accelerator is optional at run time
    (`_native.fast()` returns None without it), so a failure to build it is a warning and never
    stops libivc.so from being built."""
    try:
        build_pyfast(verbose)
    except Exception as e:  # noqa: BLE001 — optional accelerator; the ctypes paths cover it
        print(f"warning: per-block accelerator not built ({e}); the ctypes paths will be used",
              file=sys.stderr)
    if not force and up_to_date():
        return OUT
    from concurrent.futures import ThreadPoolExecutor
    objdir = os.path.join(os.path.dirname(OUT), "obj")
    os.makedirs(objdir, exist_ok=True)
    compile_flags = [f for f in FLAGS if f != "-shared"]
    objs = [os.path.join(objdir, os.path.splitext(f)[0] + ".o") for f in SOURCES]
    jobs = [[hipcc()] + compile_flags + FILE_FLAGS.get(f, []) + ["-c", "-o", o, os.path.join(CSRC, f)]
            for f, o in zip(SOURCES, objs)]
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "0") or 0) or os.cpu_count() or 1))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    tmp = OUT + ".tmp"
    _run([hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs, verbose)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose="-v" in sys.argv))
