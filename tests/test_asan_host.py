"""Host code under AddressSanitizer + UBSan (CPU only; GPU-side sanitizers are not available
on the pool).  libivc's host C++ (Huffman coder, argument checks, device-less failure paths)
is built with hipcc --cuda-host-only -fsanitize=address,undefined and the C oracle with clang
-fsanitize=address,undefined; tools/asan/asan_driver.py exercises both in a child process
with the clang ASan runtime preloaded.  Any sanitizer report fails the test."""
import glob
import hashlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ivclab_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/llvm/bin/clang"
SAN = ["-fsanitize=address,undefined", "-shared-libasan", "-fno-omit-frame-pointer", "-g", "-O1"]


def _runtime():
    hits = sorted(glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


@pytest.fixture(scope="module")
def asan_build(tmp_path_factory):
    if not (os.path.exists(HIPCC) and os.path.exists(CLANG) and _runtime()):
        pytest.skip("ROCm clang / ASan runtime not installed")
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    h = hashlib.sha256()
    for f in srcs + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "oracle", "ivc_oracle.c")]:
        h.update(open(f, "rb").read())
    d = os.path.join("/tmp", "ivc_asan_" + h.hexdigest()[:16])
    os.makedirs(d, exist_ok=True)
    ivc = os.path.join(d, "libivc_asan.so")
    orc = os.path.join(d, "liboracle_asan.so")
    if not os.path.exists(ivc):
        # device code as in the product build; every sanitizer flag goes to the host side only
        host = [x for f in SAN for x in ("-Xarch_host", f)]
        objs, procs = [], []
        for src in srcs:
            o = os.path.join(d, os.path.basename(src) + ".o")
            objs.append(o)
            procs.append(subprocess.Popen([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-c",
                                           "-ffp-contract=off", "-fno-fast-math", *host, "-o", o, src],
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        for pr in procs:
            out, _ = pr.communicate()
            assert pr.returncode == 0, out.decode()[-2000:]
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-fsanitize=address,undefined",
                        "-shared-libasan", "-o", ivc + ".tmp", *objs], check=True, capture_output=True)
        os.replace(ivc + ".tmp", ivc)
    if not os.path.exists(orc):
        subprocess.run([CLANG, "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", *SAN,
                        "-o", orc + ".tmp", os.path.join(ROOT, "oracle", "ivc_oracle.c")],
                       check=True, capture_output=True)
        os.replace(orc + ".tmp", orc)
    return ivc, orc


def test_host_code_under_asan_ubsan(asan_build):
    ivc, orc = asan_build
    env = dict(os.environ, LD_PRELOAD=_runtime(),
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=66",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=67",
               HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan", "asan_driver.py"), ivc, orc],
                       env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "asan driver: clean" in r.stdout
