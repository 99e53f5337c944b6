"""The kernels' DCT arithmetic (ivclab_amd/csrc/ivc_math.h), compiled for the host with the
same no-contraction rule, against the oracle (scipy/pocketfft) — bit for bit.  This checks
the op sequences themselves on CPU; tests/test_gpu_parity.py checks the gfx950 build."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import ivc_oracle as O
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("harness") / "harness.so")
    src = os.path.join(ROOT, "tests", "cpu_math_harness.cpp")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                    "-o", so, src], check=True)
    L = ctypes.CDLL(so)
    P = ctypes.c_void_p
    L.h_dct_f64.argtypes = [P, P, ctypes.c_long, ctypes.c_int, ctypes.c_double, ctypes.c_int]
    L.h_dct_f32.argtypes = [P, P, ctypes.c_long, ctypes.c_int, ctypes.c_float, ctypes.c_int]
    L.h_dct2_int_factored.argtypes = [P, P, ctypes.c_long]
    return L


def _run(L, fn, x, *args):
    out = np.empty_like(x)
    getattr(L, fn)(x.ctypes.data, out.ctypes.data, x.shape[0], *args)
    return out


FCT = {("ortho", 0): 0.25, ("ortho", 1): 0.25, (None, 0): 1.0, (None, 1): 1 / 16,
       ("forward", 0): 1 / 16, ("forward", 1): 1.0}


@pytest.mark.parametrize("norm", ["ortho", None, "forward"])
@pytest.mark.parametrize("inverse", [0, 1])
def test_literal_sequence_f64(harness, norm, inverse):
    rng = np.random.default_rng(10 + inverse)
    x = np.concatenate([rng.normal(0, 100, (4000, 8, 8)),
                        rng.integers(0, 256, (2000, 8, 8)).astype(np.float64),
                        np.repeat(rng.integers(-999, 999, (1000, 1, 1)), 64).reshape(1000, 8, 8) * 1.0])
    got = _run(harness, "h_dct_f64", x, inverse, FCT[(norm, inverse)], int(norm == "ortho"))
    want = O.dct_inverse(x, norm) if inverse else O.dct_transform(x, norm)
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize("inverse", [0, 1])
def test_literal_sequence_f32(harness, inverse):
    rng = np.random.default_rng(20 + inverse)
    x = rng.normal(0, 100, (5000, 8, 8)).astype(np.float32)
    got = _run(harness, "h_dct_f32", x, inverse, 0.25, 1)
    want = O.dct_inverse(x) if inverse else O.dct_transform(x)
    assert want.dtype == np.float32 and got.tobytes() == want.tobytes()


def test_factored_integer_form(harness, golden):
    """The fused kernels' factored DCT-II on integer pixels/residuals equals scipy."""
    rng = np.random.default_rng(3)
    x = np.concatenate([golden("dct")["x_u8"].astype(np.int32),
                        rng.integers(0, 256, (20000, 8, 8)),
                        rng.integers(-255, 256, (20000, 8, 8)),
                        np.repeat(rng.integers(0, 256, (2000, 1, 1)), 64).reshape(2000, 8, 8)]).astype(np.int32)
    out = np.empty(x.shape, np.float64)
    harness.h_dct2_int_factored(x.ctypes.data, out.ctypes.data, x.shape[0])
    assert out.tobytes() == O.dct_transform(x.astype(np.float64)).tobytes()
