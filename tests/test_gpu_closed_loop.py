"""The chapter-4 closed-loop video codec (exercises/ch4/ex1.py:9-373, the reference's only
working P-frame path) through the drop-in, against the same loop built from oracle
primitives (tests/closed_loop.py restates the loop once; both runs use it).

The drop-in run happens in a fresh interpreter with only the repository on PYTHONPATH (no
prelude) and the exercise's own import block (ex1.py:1-6), so every primitive is resolved by the names
the exercise uses: IntraCodec (GPU DCT / quantiser / zig-zag / zero-run, host Huffman),
MotionCompensator (GPU float64 NumPy-semantics search and block copy), rgb2ycbcr /
ycbcr2rgb (GPU colour kernels), stats_marg (GPU histogram), HuffmanCoder.  Every frame's
RGB output, the decoder's float64 YCbCr state and the motion vectors must equal the oracle
loop's bit for bit (ME runs on the decoder's reconstruction, so one differing bit anywhere
propagates into every later frame).  Bit counts: each coded message's Huffman bits lie
within [n H, n (H + 1)) of its own histogram's entropy H (bitstreams are not pinned:
constriction is absent)."""
import json
import os
import subprocess
import sys
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import closed_loop  # noqa: E402

SCALES = [0.5, 2.0]
SR = 4                       # the exercise's search range (ex1.py:392)

DROPIN = """
import json, sys
import numpy as np
from ivclab.image import IntraCodec
from ivclab.entropy import HuffmanCoder, stats_marg
from ivclab.signal import rgb2ycbcr, ycbcr2rgb
from ivclab.video import MotionCompensator
from ivclab.utils import imread, calc_psnr
sys.path.insert(0, {tests!r})
import closed_loop
from types import SimpleNamespace
api = SimpleNamespace(IntraCodec=IntraCodec, MotionCompensator=MotionCompensator,
                      rgb2ycbcr=rgb2ycbcr, ycbcr2rgb=ycbcr2rgb, stats_marg=stats_marg,
                      HuffmanCoder=HuffmanCoder, bits=True)
frames = np.load({frames!r})
summary = []
for q in {scales!r}:
    res = closed_loop.run(api, frames, q, {sr})
    for n, r in enumerate(res):
        np.save(f"{{OUT}}/rgb_{{q}}_{{n}}.npy", r["rgb"])
        np.save(f"{{OUT}}/state_{{q}}_{{n}}.npy", r["state"])
        if r["mv"] is not None:
            np.save(f"{{OUT}}/mv_{{q}}_{{n}}.npy", r["mv"])
        for k, (bits, pmf, nsym) in enumerate(r["bits"]):
            np.save(f"{{OUT}}/pmf_{{q}}_{{n}}_{{k}}.npy", pmf)
        summary.append({{"q": q, "n": n, "bits": [b for b, _, _ in r["bits"]],
                        "nsym": [m for _, _, m in r["bits"]],
                        "psnr": float(calc_psnr(frames[n], r["rgb"]))}})
print(json.dumps(summary))
"""


class _OracleIntra:
    """IntraCodec (intracodec.py:32-146) on oracle primitives, Huffman omitted (its encode /
    decode round trip is lossless; the drop-in run checks that it is)."""

    def __init__(self, quantization_scale=1.0, bounds=None, end_of_block=4000, block_shape=(8, 8)):
        self.q, self.eob = quantization_scale, end_of_block

    def image2symbols(self, img, is_source_rgb=True):
        from oracle import ivc_oracle as O
        x = O.rgb2ycbcr_fma(img) if is_source_rgb else img
        if x.ndim == 2:
            x = x[:, :, None]
        zz = O.intra_encode(x, self.q, zigzag=True)
        return O.zerorun_encode_fast(zz.reshape(-1, 64), self.eob)

    def symbols2image(self, symbols, shape):
        from oracle import ivc_oracle as O
        H, W = shape[:2]
        C = 1 if len(shape) == 2 else shape[2]
        dec = O.zerorun_decode(list(symbols), (H // 8, W // 8, C), self.eob)
        y = O.unpatch(O.intra_decode(dec, self.q, unzigzag=True))
        if C == 1:
            return y[:, :, 0] if y.shape[2] == 1 else y
        return O.ycbcr2rgb(y)

    def train_huffman_from_image(self, img, is_source_rgb=True):
        return None

    def encode_decode(self, img, is_source_rgb=True):
        return self.symbols2image(self.image2symbols(img, is_source_rgb), img.shape), None, None


class _OracleMC:
    def __init__(self, search_range=4):
        self.sr = search_range

    def compute_motion_vector(self, ref, cur):
        from oracle import ivc_oracle as O
        return O.motion_vectors(np.asarray(ref), np.asarray(cur), self.sr)

    def reconstruct_with_motion_vector(self, ref, mv):
        from oracle import ivc_oracle as O
        return O.motion_compensate(np.asarray(ref), mv, self.sr)


def _oracle_api():
    from oracle import ivc_oracle as O
    return SimpleNamespace(IntraCodec=_OracleIntra, MotionCompensator=_OracleMC,
                           rgb2ycbcr=O.rgb2ycbcr_fma, ycbcr2rgb=O.ycbcr2rgb, bits=False)


def test_ch4_closed_loop_through_dropin(tmp_path):
    frames = closed_loop.synthetic_sequence(F=8, H=64, W=80)
    np.save(tmp_path / "frames.npy", frames)
    code = f"OUT = {str(tmp_path)!r}\n" + DROPIN.format(tests=os.path.join(ROOT, "tests"),
                                                         frames=str(tmp_path / "frames.npy"),
                                                         scales=SCALES, sr=SR)
    r = subprocess.run([sys.executable, "-c", code], cwd=str(tmp_path), capture_output=True,
                       text=True, timeout=600, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(summary) == len(SCALES) * len(frames)
    oracle = _oracle_api()
    for q in SCALES:
        want = closed_loop.run(oracle, frames, q, SR)
        for n, w in enumerate(want):
            got_state = np.load(tmp_path / f"state_{q}_{n}.npy")
            assert got_state.dtype == w["state"].dtype == np.float64
            assert got_state.tobytes() == w["state"].tobytes(), f"decoder state q={q} frame {n}"
            got_rgb = np.load(tmp_path / f"rgb_{q}_{n}.npy")
            assert got_rgb.tobytes() == w["rgb"].tobytes(), f"RGB output q={q} frame {n}"
            if n:
                got_mv = np.load(tmp_path / f"mv_{q}_{n}.npy")
                assert np.array_equal(got_mv, w["mv"]) and got_mv.dtype == np.int64, f"mv q={q} frame {n}"
            # calc_psnr of the drop-in run = the oracle loop's PSNR.  It sits near 15 dB: the
            # exercise codes the 2-D luma through IntraCodec, which quantises C = 1 into 3
            # planes and decodes h*w*1 blocks of that 3-plane stream (intracodec.py:109-138),
            # a reference quirk both runs keep
            s = next(x for x in summary if x["q"] == q and x["n"] == n)
            mse = np.mean((frames[n].astype(np.float64) - w["rgb"]) ** 2)
            assert s["psnr"] == float(20 * np.log10(255 / np.sqrt(mse)))
    # the loop really searches: the P-frames' vectors vary
    mvs = np.concatenate([np.load(tmp_path / f"mv_{SCALES[0]}_{n}.npy").ravel() for n in range(1, len(frames))])
    assert len(np.unique(mvs)) > 3
    # bits: Huffman on each message's own histogram is within one bit per symbol of its entropy
    for s in summary:
        for k, (bits, n_msg) in enumerate(zip(s["bits"], s["nsym"])):
            p = np.load(tmp_path / f"pmf_{s['q']}_{s['n']}_{k}.npy")
            p = p / p.sum()
            ent = -np.sum(p * np.log2(p))
            assert n_msg * ent - 1e-6 <= bits < n_msg * (ent + 1) + 1e-6, (s, k, bits, n_msg, ent)
    # coarser quantisation spends fewer residual bits on every P-frame
    for n in range(1, len(frames)):
        b = [next(x for x in summary if x["q"] == q and x["n"] == n)["bits"][1] for q in SCALES]
        assert b[0] > b[1]

