"""CPU-side checks of the boundary: libivc.so loads, exports every symbol include/ivc.h
declares, the Python mirror keeps the reference's signatures and fails loudly (no CPU
fallback) when no gfx950 device is present."""
import inspect
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build_lib():
    from ivclab_amd import build
    return build.build()


@pytest.fixture(scope="module")
def lib():
    _build_lib()
    from ivclab_amd import _native as N
    return N.load_library()


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ivc.h")).read()
    decl = r"^\s*(?:int|int64_t|double|void\s*\*|const char\s*\*)\s*(ivc_[a-z0-9_]+)\s*\("
    return sorted(set(re.findall(decl, src, re.M)))


def test_header_symbols_exported(lib):
    import ivclab_amd._native as N
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"libivc.so does not export {s}"
    assert set(syms) == set(N.EXPORTS), "ctypes signature table out of sync with include/ivc.h"


def test_nm_shows_gfx950_code_object(lib):
    from ivclab_amd import build
    data = open(build.OUT, "rb").read()
    assert b"gfx950" in data


def test_no_device_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from ivclab_amd import _native as N
    from ivclab_amd.signal import DiscreteCosineTransform
    assert lib.ivc_device_count() == 0
    with pytest.raises(N.IvcError, match="no CPU fallback"):
        DiscreteCosineTransform().transform(np.zeros((8, 8)))


def test_status_mapping(lib):
    from ivclab_amd import _native as N
    # a bad dtype code fails argument validation before any device work
    rc = lib.ivc_quantize(None, 99, 1, 1, None, 10, None)
    assert rc == N.E_DTYPE
    with pytest.raises(ValueError, match="invalid source dtype"):
        N.check(rc, "quantize")
    rc = lib.ivc_motion_estimate(None, None, 10, 1, 12, 16, 4, 0, None)
    assert rc == N.E_SHAPE
    assert b"multiples of 8" in lib.ivc_last_error()


def test_reference_signatures():
    """Same constructor parameters and methods as the reference classes."""
    import ivclab_amd as IA
    from ivclab_amd.signal.zigzag import zigzag_scan
    sig = lambda f: list(inspect.signature(f).parameters)  # noqa: E731
    assert sig(IA.DiscreteCosineTransform.__init__) == ["self", "norm"]
    assert IA.DiscreteCosineTransform().norm == "ortho"
    assert sig(IA.PatchQuant.__init__) == ["self", "quantization_scale", "luminance", "chrominance"]
    q = IA.PatchQuant()
    assert q.quantization_scale == 1.0 and q.luminance.dtype == np.float32
    assert sig(IA.MotionCompensator.__init__) == ["self", "search_range"]
    assert IA.MotionCompensator().search_range == 4
    assert sig(IA.Patcher.__init__) == ["self", "window_size"]
    assert sig(zigzag_scan) == ["block"]
    for cls, meths in ((IA.DiscreteCosineTransform, ["transform", "inverse_transform"]),
                       (IA.PatchQuant, ["get_quantization_table", "quantize", "dequantize"]),
                       (IA.ZigZag, ["flatten", "unflatten"]), (IA.Patcher, ["patch", "unpatch"]),
                       (IA.MotionCompensator, ["compute_motion_vector",
                                               "reconstruct_with_motion_vector"])):
        for m in meths:
            assert callable(getattr(cls, m))


def test_host_logic_tables_and_layout(golden):
    """Host-side pieces that need no device: table construction and patch views."""
    import ivclab_amd as IA
    from oracle import ivc_oracle as O
    q = golden("quant")
    for i, s in enumerate(q["scales"]):
        t = IA.PatchQuant(float(s)).get_quantization_table()
        assert t.dtype == q[f"table_{i}"].dtype and t.tobytes() == q[f"table_{i}"].tobytes()
    img = q["img3"]
    assert np.array_equal(IA.Patcher().patch(img), O.patch(img))
    assert np.array_equal(IA.Patcher().unpatch(IA.Patcher().patch(img)), img)
    assert np.array_equal(IA.ZigZag().zigzag_order, O.ZZ_ORDER)
    from ivclab_amd.quantization.patchquant import _as_blocks
    src, C, shp = _as_blocks(np.zeros((4, 5, 1, 8, 8)), t)
    assert C == 1 and shp == (4, 5, 3, 8, 8)
    src, C, shp = _as_blocks(np.zeros((8, 8)), t)
    assert C == 1 and shp == (1, 1, 3, 8, 8)
    src, C, shp = _as_blocks(np.zeros((1, 8)), t)
    assert C == 3 and shp == (1, 1, 3, 8, 8) and src.shape == shp
    with pytest.raises(ValueError):
        _as_blocks(np.zeros((2, 8, 8)), t)


def test_install_as_ivclab():
    import sys

    import ivclab_amd as IA
    for k in [k for k in sys.modules if k == "ivclab" or k.startswith("ivclab.")]:
        del sys.modules[k]
    assert IA.install_as_ivclab() is sys.modules["ivclab"]
    try:
        from ivclab.quantization import PatchQuant
        from ivclab.signal import DiscreteCosineTransform
        from ivclab.signal.zigzag import zigzag_scan  # noqa: F401
        from ivclab.utils import Patcher, ZigZag  # noqa: F401
        from ivclab.utils.metrics import calc_mse
        from ivclab.video import MotionCompensator  # noqa: F401
        from ivclab.video.videocodec import VideoCodec
        assert VideoCodec is IA.VideoCodec
        assert DiscreteCosineTransform is IA.DiscreteCosineTransform
        assert PatchQuant is IA.PatchQuant
        assert calc_mse(np.zeros((2, 2, 3)), np.ones((2, 2, 3))) == 1.0
    finally:
        for k in [k for k in sys.modules if k == "ivclab" or k.startswith("ivclab.")]:
            del sys.modules[k]


def test_single_hip_runtime_with_torch(lib):
    """libivc and torch must share one HIP runtime (two runtimes cannot both own the GPU)."""
    import torch  # noqa: F401
    maps = open("/proc/self/maps").read().splitlines()
    hips = {ln.split()[-1] for ln in maps if "libamdhip64" in ln}
    assert len(hips) == 1, hips


def test_symbol_pmf_from_counts_matches_stats_marg():
    """The host finish of the Huffman-table input (counts from the GPU histogram) equals
    the reference's stats_marg + smooth_pmf on the symbol stream itself, bit for bit."""
    from oracle import ivc_oracle as O
    from ivclab_amd.entropy.stats import huffman_bounds, smooth_pmf, stats_marg_from_counts
    rng = np.random.default_rng(9)
    sym = np.concatenate([rng.integers(-60, 61, 20000), np.full(3000, 4000), [0] * 5000]).astype(np.int32)
    b0, b1 = huffman_bounds(sym.min(), sym.max())
    counts = O.histogram(sym, b0, b1 - b0 - 1)        # what ivc_histogram_i32 returns
    got = smooth_pmf(stats_marg_from_counts(counts))
    want = O.smooth_pmf(O.stats_marg(sym, np.arange(b0, b1)))
    assert got.dtype == want.dtype and got.tobytes() == want.tobytes()


def test_huffman_host_coder():
    """libivc's host Huffman coder (no device needed): the reference module's own example
    (huffman.py:55-61: 29 bits, exact round trip), the reference's errors, optimality on a
    large alphabet (bit count = sum of code lengths, within 1 bit/symbol of the entropy)."""
    from ivclab_amd.entropy import HuffmanCoder
    h = HuffmanCoder(lower_bound=0)
    with pytest.raises(RuntimeError):
        h.encode(np.array([0]))
    probs = np.array([0.5, 0.25, 0.25], dtype=np.float32)
    msg = np.array([0, 2, 1, 2, 1, 0, 2, 0, 1, 0, 0, 2, 2, 0, 1, 0, 0, 2, 0])
    h.train(probs)
    comp, bits = h.encode(msg)
    assert bits == 29.0
    assert np.array_equal(h.decode(comp, len(msg)), msg)
    assert h.is_prefix_free()
    with pytest.raises(ValueError, match="outside the trained range"):
        h.encode(np.array([3]))
    with pytest.raises(ValueError, match="Zero-probability"):
        HuffmanCoder().train(np.array([0.5, 0.0, 0.5]))
    rng = np.random.default_rng(5)
    p = rng.random(4000) ** 4 + 1e-9
    p /= p.sum()
    h2 = HuffmanCoder(lower_bound=-1000)
    h2.train(p)
    m = rng.choice(np.arange(-1000, 3000), size=300000, p=p)
    comp, bits = h2.encode(m)
    assert np.array_equal(h2.decode(comp, m.size), m)
    L = h2.encoder_codebook.astype(np.float64)
    assert bits == L[m + 1000].sum()
    H = -(p * np.log2(p)).sum()
    assert H <= (p * L).sum() < H + 1


def test_pmc_record_key_matches_bench():
    """The committed HBM-traffic record (profiles/pmc_intra_latest.json) is keyed by the HIP
    source hash that bench.py computes; tools/pmc_traffic.py writes the same key."""
    import importlib.util
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mods = {}
    for name, path in (("bench", "bench.py"), ("pmc_traffic", "tools/pmc_traffic.py")):
        spec = importlib.util.spec_from_file_location("_t_" + name, os.path.join(root, path))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        mods[name] = m
    key = mods["bench"].csrc_sha256()
    assert key == mods["pmc_traffic"].csrc_sha256() and len(key) == 64
    rec = json.load(open(os.path.join(root, "profiles", "pmc_intra_latest.json")))
    assert {"hbm_bytes_per_launch", "frames", "H", "W", "csrc_sha256"} <= set(rec)
    assert 0.99 < rec["hbm_bytes_per_launch"] / rec["algorithmic_bytes_per_launch"] < 1.05


def test_device_barriers_drain_lds():
    """Every workgroup barrier in the device sources goes through ivc::lds_barrier (an
    lgkmcnt(0) wait, then the barrier): hipcc omits that wait at some loop-header barriers and
    on gfx950 another wave can then read a stale LDS word (ivc_internal.h; the compiled-code
    check is tools/check_barriers.py)."""
    csrc = os.path.join(ROOT, "ivclab_amd", "csrc")
    offenders = []
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".hip", ".h")):
            continue
        with open(os.path.join(csrc, name)) as f:
            for n, line in enumerate(f, 1):
                code = line.split("//")[0]
                if re.search(r"__syncthreads\s*\(|__builtin_amdgcn_s_barrier\s*\(", code) and \
                        "asm volatile(\"s_waitcnt lgkmcnt(0)\"" not in code:
                    offenders.append(f"{name}:{n}")
    # the one raw barrier is lds_barrier's own
    assert offenders == ["ivc_internal.h:" + str(_lds_barrier_line(csrc))], offenders


def _lds_barrier_line(csrc):
    with open(os.path.join(csrc, "ivc_internal.h")) as f:
        lines = f.read().split("\n")
    start = next(i for i, l in enumerate(lines) if "void lds_barrier()" in l)
    return next(i for i in range(start, start + 4) if "__syncthreads()" in lines[i]) + 1
