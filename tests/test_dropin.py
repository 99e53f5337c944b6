"""The drop-in boundary seen from the reference's own callers: with only this repository on
PYTHONPATH (no prelude, no install step, a scratch working directory) the import lines of
the reference's tests and chapter 3/4 exercises resolve unchanged to the repository's own
`ivclab` package, and tests/ch3.py's assertions (tests/ch3.py:18-47) hold on a committed
synthetic stand-in for the absent data/satpic1.bmp with the thresholds the reference itself
computes on that image (tests/golden/ch3.npz, make_golden.py make_ch3).

The import checks run in a fresh interpreter and need no GPU: importing the drop-in loads
libivc lazily.  The ch3 assertions compute on the GPU."""
import ast
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
STANDIN = os.path.join(ROOT, "tests", "golden", "satpic_standin.bmp")

# tests/ch3.py:1-8, the reference's API-contract test, verbatim import block
CH3_IMPORTS = """\
import unittest
import numpy as np
from ivclab.utils import imread
from ivclab.utils import Patcher
from ivclab.signal import DiscreteCosineTransform
from ivclab.quantization import PatchQuant
from ivclab.utils import calc_psnr
from ivclab.utils.metrics import calc_mse
"""


def caller_env():
    """The caller's environment: PYTHONPATH = this repository and nothing else of ours."""
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT
    return env


def run_py(code, cwd=None):
    """Run `code` as an unchanged caller would: a fresh interpreter, the repository only on
    PYTHONPATH, started from a directory outside it."""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([sys.executable, "-c", code], cwd=cwd or d, env=caller_env(),
                           capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def test_ch3_import_block_resolves():
    out = run_py(CH3_IMPORTS + "import ivclab, os\n"
                 "print(imread.__module__, Patcher.__module__, calc_mse.__module__)\n"
                 "print(os.path.dirname(os.path.dirname(ivclab.__file__)))")
    lines = out.splitlines()
    assert lines[0].split() == ["ivclab_amd.utils.io", "ivclab_amd.utils.shape",
                                "ivclab_amd.utils.metrics"]
    assert lines[1] == ROOT


def test_package_layout_mirrors_reference():
    """ivclab/__init__.py:1-5 star-imports entropy, image, quantization, utils, video (not
    signal); the subpackages export the hot-path names; `import ivclab` needs no
    constriction; names outside the hot path raise ImportError."""
    out = run_py("""
import sys, ivclab
assert 'constriction' not in sys.modules
for n in ('PatchQuant', 'ZigZag', 'Patcher', 'imread', 'calc_psnr', 'calc_mse', 'IntraCodec',
          'MotionCompensator', 'VideoCodec', 'HuffmanCoder', 'ZeroRunCoder', 'stats_marg',
          'smooth_pmf', 'calc_entropy', 'min_code_length'):
    assert hasattr(ivclab, n), n
assert not hasattr(ivclab, 'DiscreteCosineTransform')   # signal is not star-imported
import ivclab.signal.zigzag, ivclab.utils.shape, ivclab.video.motion, ivclab.entropy.entropy
assert ivclab.signal.zigzag.zigzag_scan.__module__ == 'ivclab_amd.signal.zigzag'
assert not hasattr(ivclab.signal, 'zigzag_scan')       # signal/__init__.py does not export it
import ivclab_amd
assert ivclab.signal.DiscreteCosineTransform is ivclab_amd.DiscreteCosineTransform
assert ivclab.video.videocodec.VideoCodec is ivclab_amd.VideoCodec
for mod, name in (('ivclab.signal', 'downsample'), ('ivclab.signal', 'FilterPipeline'),
                  ('ivclab.image', 'IntraCodecAdaptive'), ('ivclab.entropy', 'stats_joint')):
    try:
        exec(f'from {mod} import {name}')
    except ImportError as e:                 # the reason reaches the from-import form too
        assert 'outside the MI355X block-codec hot path' in str(e), (name, str(e))
    else:
        raise AssertionError(name)
try:
    ivclab.signal.downsample
except AttributeError as e:               # attribute access: the reason, as an AttributeError
    assert 'outside the MI355X block-codec hot path' in str(e)
else:
    raise AssertionError('downsample')
assert hasattr(ivclab.signal, 'downsample') is False       # probes behave as on absent names
assert getattr(ivclab.image, 'IntraCodecAdaptive', 7) == 7
import ivclab.signal as S
try:
    from ivclab.signal import FilterPipeline as _fp       # from-import of a package attribute
except ImportError as e:
    assert 'outside the MI355X block-codec hot path' in str(e)
else:
    raise AssertionError('FilterPipeline')
try:
    ivclab.signal.no_such_name
except AttributeError as e:
    assert 'outside' not in str(e)
print('ok')
""")
    assert out.strip() == "ok"


def _reference_import_lines():
    """Every `from ivclab... import ...` / `import ivclab...` statement of the reference's
    tests/ch3.py and exercises/ch3, ch4 (the chapters whose hot path this build covers)."""
    files = [os.path.join(REF, "tests", "ch3.py")]
    files += sorted(glob.glob(os.path.join(REF, "exercises", "ch3", "*.py")))
    files += sorted(glob.glob(os.path.join(REF, "exercises", "ch4", "*.py")))
    stmts = set()
    for f in files:
        tree = ast.parse(open(f).read())
        for node in ast.walk(tree):
            if isinstance(node, ast.ImportFrom) and (node.module or "").startswith("ivclab"):
                stmts.add(f"from {node.module} import " + ", ".join(a.name for a in node.names))
            elif isinstance(node, ast.Import):
                for a in node.names:
                    if a.name.startswith("ivclab"):
                        stmts.add(f"import {a.name}")
    return sorted(stmts)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_reference_callers_import_lines_resolve():
    stmts = _reference_import_lines()
    assert len(stmts) >= 10
    code = "\n".join(stmts) + "\nprint('ok')"
    assert run_py(code).strip() == "ok"


def test_imread_matches_pil():
    from PIL import Image
    from ivclab_amd.utils import imread
    img = imread(STANDIN)
    with Image.open(STANDIN) as im:
        want = np.asarray(im)
    assert img.dtype == np.uint8 and img.shape == (256, 256, 3)
    assert np.array_equal(img, want)


@pytest.mark.gpu
def test_ch3_assertions_on_standin(golden):
    """tests/ch3.py:18-47 through the drop-in names, on the stand-in image: the same
    assertions and deltas, with the expected values the reference computes for this image
    (and, tighter, equal to them: the path is bit-exact)."""
    code = CH3_IMPORTS + f"""
import json
orig_img = imread({STANDIN!r})
patcher = Patcher(window_size=(8, 8))
dct = DiscreteCosineTransform(norm='ortho')
quantizer = PatchQuant(quantization_scale=1.0)
patched_img = patcher.patch(orig_img)
transformed = dct.transform(patched_img)
reconstructed_patched = dct.inverse_transform(transformed)
quantized = quantizer.quantize(patched_img)
dequantized = quantizer.dequantize(quantized)
reconstructed = patcher.unpatch(dequantized)
print(json.dumps({{"mean_energy": float(np.mean(transformed ** 2)),
                  "inverse_allclose": bool(np.allclose(reconstructed_patched, patched_img)),
                  "mean_q2": float(np.mean(quantized ** 2)),
                  "mse": float(calc_mse(orig_img, reconstructed)),
                  "psnr": float(calc_psnr(orig_img, reconstructed))}}))
"""
    import json
    got = json.loads(run_py(code).strip().splitlines()[-1])
    want = golden("ch3")
    assert abs(got["mean_energy"] - want["mean_energy"]) <= 100          # ch3.py:21
    assert got["inverse_allclose"]                                       # ch3.py:27
    assert abs(got["mean_q2"] - want["mean_q2"]) <= 0.1                  # ch3.py:40
    assert abs(got["mse"] - want["mse"]) <= 5                            # ch3.py:47
    for k in ("mean_energy", "mean_q2", "mse", "psnr"):
        assert got[k] == float(want[k]), k


# exercises/ch3/ex1.py's rate-distortion loop (its quantisation scales, Huffman trained on a
# small training image with is_source_rgb=False, the large image coded and decoded), through
# the drop-in names on synthetic stand-ins for the absent data/lena.tif / lena_small.tif
RD_SCALES = [0.05, 0.1, 0.15, 0.2, 0.3]
RD_CODE = """
import json
import numpy as np
from ivclab.image import IntraCodec
from ivclab.utils import calc_psnr
rng = np.random.default_rng(31)
yy, xx = np.mgrid[0:256, 0:384]
base = 128 + 60 * np.sin(xx / 23.0) * np.cos(yy / 17.0) + 0.2 * (xx - yy)
lena = np.stack([base + 25 * np.sin(yy / (7.0 + 3 * c)) for c in range(3)], axis=-1)
lena = np.clip(lena + rng.normal(0, 6, lena.shape), 0, 255).astype(np.uint8)
lena_small = np.ascontiguousarray(lena[::2, ::2])
rows = []
for q in %r:
    codec = IntraCodec(quantization_scale=q)
    codec.train_huffman_from_image(lena_small, is_source_rgb=False)
    rec, bitstream, bitsize, bpp = codec.encode_decode(lena, return_bpp=True, is_source_rgb=False)
    syms = codec.image2symbols(lena, is_source_rgb=False)
    np.save(f"{OUT}/rec_{q}.npy", rec)
    np.save(f"{OUT}/sym_{q}.npy", np.asarray(syms, np.int32))
    np.save(f"{OUT}/len_{q}.npy", np.asarray(codec.huffman.encoder_codebook, np.int64))
    np.save(f"{OUT}/pmf_{q}.npy", np.asarray(codec.huffman.probs, np.float64))
    rows.append({"q": q, "psnr": float(calc_psnr(lena, rec)), "bits": int(bitsize), "bpp": float(bpp),
                 "bounds": list(codec.bounds)})
np.save(f"{OUT}/lena.npy", lena)
print(json.dumps(rows))
"""


@pytest.mark.gpu
def test_exercise_ch3_rd_curve(tmp_path):
    """exercises/ch3/ex1.py's RD loop through the drop-in: every reconstruction equals the
    oracle chain (patch -> DCT -> quantise -> zig-zag -> zero-run -> decode -> dequantise ->
    IDCT -> unpatch -> ycbcr2rgb) bit for bit, so every PSNR is the reference's; the symbol streams equal
    the oracle's.  Bitrates (bitstreams are not pinned: constriction's tie-breaking is
    absent): the bit count is the sum of the coder's code lengths over the stream, the
    lengths are a complete prefix code (Kraft sum 1) within the Huffman bound on the trained
    pmf (mean length < H(pmf) + 1), and no prefix code spends fewer bits than the stream's
    empirical entropy.  The bitrate falls as the scale grows."""
    import json
    sys.path.insert(0, ROOT)
    from oracle import ivc_oracle as O
    code = f"OUT = {str(tmp_path)!r}\n" + RD_CODE % (RD_SCALES,)
    rows = json.loads(run_py(code).strip().splitlines()[-1])
    lena = np.load(tmp_path / "lena.npy")
    H, W, _ = lena.shape
    for r in rows:
        q = r["q"]
        zz = O.intra_encode(lena, q, zigzag=True)
        want_sym = O.zerorun_encode_fast(zz.reshape(-1, 64))
        got_sym = np.load(tmp_path / f"sym_{q}.npy")
        assert np.array_equal(got_sym, want_sym), f"symbols q={q}"
        dec = O.zerorun_decode(want_sym, (H // 8, W // 8, 3))
        # symbols2image of a 3-D shape ends in ycbcr2rgb, even for is_source_rgb=False input
        # (intracodec.py:140-146, the reference's behaviour)
        want_rec = O.ycbcr2rgb(O.unpatch(O.intra_decode(dec, q, unzigzag=True)))
        rec = np.load(tmp_path / f"rec_{q}.npy")
        assert rec.dtype == want_rec.dtype and rec.shape == want_rec.shape
        assert rec.tobytes() == want_rec.tobytes(), f"reconstruction q={q}"
        assert r["psnr"] == float(20 * np.log10(255 / np.sqrt(np.mean((lena.astype(np.float64) - want_rec) ** 2))))
        # the trained code (intracodec.py:149-166: pmf over [min-20, max+21), smoothed)
        lo = r["bounds"][0]
        ln = np.load(tmp_path / f"len_{q}.npy")
        pmf = np.load(tmp_path / f"pmf_{q}.npy")
        assert r["bits"] == int(ln[want_sym - lo].sum())
        assert abs(np.sum(2.0 ** -ln.astype(np.float64)) - 1.0) < 1e-12
        h = -np.sum(pmf * np.log2(pmf))
        assert np.sum(pmf * ln) < h + 1
        e = np.bincount(want_sym - want_sym.min()).astype(np.float64)
        e = e[e > 0] / len(want_sym)
        assert r["bits"] >= len(want_sym) * -np.sum(e * np.log2(e)) - 1e-6
        assert r["bpp"] == r["bits"] / (H * W)
    # coarser quantisation: fewer bits (PSNR is not monotone here: the reference decodes a 3-D
    # shape through ycbcr2rgb although this image was coded as YCbCr, with clipping)
    bpp = [r["bpp"] for r in rows]
    assert all(a > b for a, b in zip(bpp, bpp[1:])), rows
