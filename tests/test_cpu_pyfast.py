"""The per-block call accelerator (ivclab_amd/csrc/ivc_pyfast.c) on the CPU: its eligibility
rules, output shapes and dtypes and argument passing, with stand-in entry points (ctypes
callbacks that record their arguments) in place of libivc's."""
import ctypes as ct
import importlib.machinery
import importlib.util
import os
import sysconfig

import numpy as np
import pytest

from ivclab_amd.quantization.patchquant import _fast_args

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "ivclab_amd", "_lib", "_ivcfast" + sysconfig.get_config_var("EXT_SUFFIX"))

DCT = ct.CFUNCTYPE(ct.c_int, ct.c_void_p, ct.c_int, ct.c_int64, ct.c_void_p, ct.c_int, ct.c_int, ct.c_int)
QNT = ct.CFUNCTYPE(ct.c_int, ct.c_void_p, ct.c_int, ct.c_int64, ct.c_int, ct.c_void_p, ct.c_int, ct.c_void_p)


@pytest.fixture(scope="module")
def fast():
    if not os.path.exists(PATH):
        pytest.skip("accelerator not built")
    loader = importlib.machinery.ExtensionFileLoader("pyfast_standin._ivcfast", PATH)
    spec = importlib.util.spec_from_file_location("pyfast_standin._ivcfast", PATH, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    calls, tabs = [], []

    def dct(src, code, nblk, dst, ocode, inv, norm):
        calls.append(("dct", code, nblk, ocode, inv, norm))
        return 0

    def qnt(which):
        def f(src, code, nblk, C, tab, cc, dst):
            calls.append((which, code, nblk, C, tab, cc))
            tabs.append(np.ctypeslib.as_array(ct.cast(tab, ct.POINTER(ct.c_double)), (192,)).copy()
                        if tab > 4096 else None)
            return 7 if nblk == 5 else 0          # a failing call returns its status
        return f

    cbs = [DCT(dct), QNT(qnt("q")), QNT(qnt("dq"))]
    addr = [ct.cast(c, ct.c_void_p).value for c in cbs]
    mod.set_entry_points(*addr)
    mod._keep = cbs
    mod._tabs = tabs
    return mod, calls


def test_dct_eligibility_and_dtypes(fast):
    mod, calls = fast
    for dt, code, odt in [(np.uint8, 1, np.float64), (np.float32, 9, np.float32),
                          (np.int64, 8, np.float64), (np.float64, 10, np.float64)]:
        x = np.zeros((3, 8, 8), dt)
        r = mod.dct8x8(x, 1, 0)
        assert r.dtype == odt and r.shape == x.shape
        assert calls[-1] == ("dct", code, 3, 9 if odt == np.float32 else 10, 0, 1)
    assert mod.dct8x8(np.zeros((8, 8), np.float16), 1, 0) is None         # not a kernel dtype
    assert mod.dct8x8(np.zeros((8, 8), ">f8"), 1, 0) is None              # byte-swapped
    assert mod.dct8x8(np.zeros((16, 16))[::2, ::2], 1, 0) is None         # not contiguous
    assert mod.dct8x8(np.zeros((8, 9)), 1, 0) is None
    assert mod.dct8x8(np.zeros((0, 8, 8)), 1, 0) is None                  # empty
    assert mod.dct8x8(np.zeros((65, 8, 8)), 1, 0) is None                 # over 4096 elements
    assert mod.dct8x8(np.zeros(64), 1, 0) is None


@pytest.mark.parametrize("shape", [(8, 8), (3, 8, 8), (1, 8, 8), (4, 3, 8, 8), (2, 4, 1, 8, 8),
                                   (1, 2, 2, 3, 8, 8)])
def test_quant_shapes_match_the_python_fast_path(fast, shape):
    mod, calls = fast
    x = np.zeros(shape, np.float64)
    for xdt in (np.float64, np.float32, np.uint8, np.int16, np.int32, np.uint64):
        for tdt, tcode in ((np.float64, 10), (np.float32, 9)):
            xx = x.astype(xdt)
            r = mod.quant(False, xx, 1234, tcode)
            code, C, oshape, cc = _fast_args(xx.dtype, xx.shape, np.dtype(tdt))
            assert r.shape == oshape and r.dtype == np.int32
            assert calls[-1] == ("q", code, r.size // 192, C, 1234, cc), (xdt, tdt)
    r = mod.quant(True, x.astype(np.int32), 99, 10)
    assert calls[-1][0] == "dq" and r.shape == oshape


def test_quant_rejects_and_status(fast):
    mod, calls = fast
    assert mod.quant(False, np.zeros((2, 8, 8)), 1, 10) is None           # C = 2 broadcasts
    assert mod.quant(False, np.zeros((8, 8), np.complex128), 1, 10) is None
    assert mod.quant(False, np.zeros((193, 8, 8)), 1, 10) is None          # over 12288 elements
    assert mod.quant(False, np.zeros((8, 8)), 1, 8) is None               # an int64 table
    assert mod.quant(False, np.zeros((5, 1, 8, 8)), 1, 10) == 7           # the status comes back


def test_quant_lc_forms_numpys_table(fast):
    """quant_lc builds stack([lum, chrom, chrom]) * scale itself (patchquant.py:39-42) whenever
    NumPy's result is a float32 or float64 table, bit for bit with the same type, and declines
    everything else."""
    from ivclab_amd.quantization.patchquant import _CHROM, _LUM
    mod, calls = fast
    rng = np.random.default_rng(3)
    lf = rng.uniform(0.1, 300, (8, 8))
    l32 = rng.uniform(0.1, 300, (8, 8)).astype(np.float32)
    li = rng.integers(1, 200, (8, 8))
    big = rng.integers(-2**62, 2**62, (8, 8))           # int64 entries that round to double
    cases = [(_LUM, _CHROM, 1.0), (_LUM, _CHROM, 0.37), (_LUM, _CHROM, 3), (_LUM, l32, 1e-7),
             (_LUM, _CHROM, np.float64(0.37)), (_LUM, _CHROM, 1e39), (_LUM, _CHROM, -2**24),
             (lf, _CHROM, 3), (lf, lf, np.float64(1e-3)), (li, li, 0.3), (li, _CHROM, 7),
             (big, _CHROM, 1.5), (li, lf, -2**53), (lf, _CHROM, float("nan"))]
    x = np.zeros((3, 8, 8), np.float32)      # float32 arithmetic exactly when the table is float32
    for lum, chrom, sc in cases:
        with np.errstate(over="ignore"):
            want = np.stack([lum, chrom, chrom], axis=0) * sc
        assert want.dtype in (np.float32, np.float64)
        r = mod.quant_lc(False, x, lum, chrom, sc)
        assert r is not None and calls[-1][0] == "q", (lum.dtype, chrom.dtype, sc)
        assert calls[-1][5] == (9 if want.dtype == np.float32 else 10), (lum.dtype, chrom.dtype, sc)
        got = mod._tabs[-1]
        np.testing.assert_array_equal(got.view(np.uint64),
                                      want.reshape(-1).astype(np.float64).view(np.uint64))
    r = mod.quant_lc(True, x.astype(np.int32), lf, lf, 2.0)
    assert calls[-1][0] == "dq" and r.shape == (1, 1, 3, 8, 8)
    n = len(calls)
    declined = [(li, li, 2),                                 # an int64 table
                (_LUM, _CHROM, np.float32(1.0)), (_LUM, _CHROM, True), (lf, _CHROM, 2**60),
                (_LUM, _CHROM, 2**24 + 1), (_LUM.astype(np.float16), _CHROM, 1.0),
                (np.ascontiguousarray(lf.T).T, lf, 1.0), (lf.astype(">f8"), lf, 1.0),
                (lf.reshape(1, 8, 8), lf, 1.0), ([[1.0] * 8] * 8, lf, 1.0),
                (li.astype(np.int32), lf, 1.0), (lf, lf, np.int64(2))]
    for lum, chrom, sc in declined:
        assert mod.quant_lc(False, x, lum, chrom, sc) is None, (lum, sc)
    assert len(calls) == n
    assert mod.quant_lc(False, np.zeros((5, 1, 8, 8)), lf, lf, 1.0) == 7
