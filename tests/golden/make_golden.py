"""Generate the golden input/output vectors for the hot path FROM THE REFERENCE ITSELF.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
It loads the reference hot-path modules by file path (the package __init__ needs the
absent `constriction` wheel, so `import ivclab` itself fails; these modules import only
numpy/scipy/einops), runs them on seeded synthetic inputs and writes small .npz fixtures
next to this script.  Only data (inputs and the reference's outputs) is committed; nothing
from the reference ships.  The GPU box never runs this script.

Reference modules used (paths relative to /root/reference):
  ivclab/signal/dct.py            DiscreteCosineTransform
  ivclab/quantization/patchquant.py PatchQuant
  ivclab/utils/shape.py           ZigZag, Patcher
  ivclab/signal/zigzag.py         zigzag_scan
  ivclab/video/motion.py          MotionCompensator
  ivclab/entropy/zerorun.py       ZeroRunCoder (zerorun.npz; its own RNG stream, so the
                                  other fixtures are unchanged by its addition)
  ivclab/signal/color.py          rgb2gray, rgb2ycbcr, ycbcr2rgb (color.npz; own RNG stream)
  ivclab/entropy/entropy.py       stats_marg, smooth_pmf, calc_entropy (stats.npz; imported as
                                  ivclab.entropy.entropy with the `ivclab` and `ivclab.entropy`
                                  package __init__ files bypassed — they import huffman.py,
                                  which needs the absent `constriction`)
  ivclab/utils/metrics.py         calc_mse, calc_psnr (ch3.npz: the quantities tests/ch3.py:18-47
                                  asserts, computed by the reference on a synthetic stand-in for
                                  the absent data/satpic1.bmp, written as satpic_standin.bmp)

    python tests/golden/make_golden.py [ch3 ...]   # only the named fixture groups
"""
import contextlib
import importlib.util
import io
import os
import sys

import numpy as np

REF = os.environ.get("IVC_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _load(rel, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _quiet(fn, *a):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a)


def blocks_u8(rng, n):
    """Mixed 8x8 uint8 content: noise, constants (DC ties), checkerboards, ramps."""
    x = rng.integers(0, 256, (n, 8, 8)).astype(np.uint8)
    k = n // 8
    x[:k] = rng.integers(0, 256, (k, 1, 1))                                   # constant
    cb = (np.indices((8, 8)).sum(0) % 2).astype(np.uint8)
    x[k:2 * k] = cb[None] * rng.integers(0, 256, (k, 1, 1)).astype(np.uint8)  # checkerboard
    ramp = np.add.outer(np.arange(8), np.arange(8))
    x[2 * k:3 * k] = (ramp[None] * rng.integers(1, 17, (k, 1, 1))).clip(0, 255)  # ramps
    x[3 * k] = 255
    x[3 * k + 1] = 0
    return x


def image_u8(rng, H, W, C):
    """Synthetic image built from the same block mix."""
    b = blocks_u8(rng, (H // 8) * (W // 8) * C)
    rng.shuffle(b)
    return b.reshape(H // 8, W // 8, C, 8, 8).transpose(0, 3, 1, 4, 2).reshape(H, W, C).copy()


def main():
    dct_m = _load("ivclab/signal/dct.py", "ref_dct")
    pq_m = _load("ivclab/quantization/patchquant.py", "ref_patchquant")
    sh_m = _load("ivclab/utils/shape.py", "ref_shape")
    zz_m = _load("ivclab/signal/zigzag.py", "ref_zigzag")
    mo_m = _load("ivclab/video/motion.py", "ref_motion")
    rng = np.random.default_rng(20250629)
    DCT = dct_m.DiscreteCosineTransform()

    # ---------------------------------------------------------------- DCT / IDCT
    d = {}
    d["x_u8"] = blocks_u8(rng, 1024)
    d["dct_u8"] = DCT.transform(d["x_u8"])
    d["x_f64"] = rng.normal(0, 60, (256, 8, 8))
    d["dct_f64"] = DCT.transform(d["x_f64"])
    d["idct_f64"] = DCT.inverse_transform(d["x_f64"])
    d["x_f32"] = rng.normal(0, 60, (256, 8, 8)).astype(np.float32)
    d["dct_f32"] = DCT.transform(d["x_f32"])
    d["idct_f32"] = DCT.inverse_transform(d["x_f32"])
    d["x_i32"] = rng.integers(-1200, 1200, (256, 8, 8)).astype(np.int32)
    d["idct_i32"] = DCT.inverse_transform(d["x_i32"])
    d["x_i16"] = rng.integers(-255, 256, (64, 8, 8)).astype(np.int16)
    d["dct_i16"] = DCT.transform(d["x_i16"])
    for norm in ("backward", "forward"):
        D2 = dct_m.DiscreteCosineTransform(norm=norm)
        d[f"dct_f64_{norm}"] = D2.transform(d["x_f64"][:64])
        d[f"idct_f64_{norm}"] = D2.inverse_transform(d["x_f64"][:64])
    d["x_img"] = image_u8(rng, 64, 48, 3)
    d["dct_img"] = DCT.transform(_quiet(sh_m.Patcher().patch, d["x_img"]))
    np.savez_compressed(os.path.join(OUT, "dct.npz"), **d)

    # ---------------------------------------------------------------- quantisation
    q = {}
    img1 = image_u8(rng, 64, 64, 1)
    img3 = image_u8(rng, 64, 64, 3)
    q["img1"], q["img3"] = img1, img3
    P = sh_m.Patcher()
    dct1 = DCT.transform(P.patch(img1))
    dct3 = DCT.transform(P.patch(img3))
    q["scales"] = np.array([1.0, 0.5, 0.15, 2.0, 0.07])
    for i, s in enumerate(q["scales"]):
        Q = pq_m.PatchQuant(quantization_scale=float(s))
        q[f"table_{i}"] = Q.get_quantization_table()
        q[f"q1_{i}"] = Q.quantize(dct1)
        q[f"q3_{i}"] = Q.quantize(dct3)
        q[f"dq1_{i}"] = Q.dequantize(q[f"q1_{i}"])
        q[f"dq3_{i}"] = Q.dequantize(q[f"q3_{i}"])
        q[f"idq3_{i}"] = DCT.inverse_transform(q[f"dq3_{i}"])
    Q1 = pq_m.PatchQuant(quantization_scale=1.0)
    q["raw_q3"] = Q1.quantize(P.patch(img3))                    # tests/ch3.py:37-40 shape
    q["raw_dq3"] = Q1.dequantize(q["raw_q3"])
    f32in = DCT.transform(P.patch(img3).astype(np.float32))
    q["f32_dct3"] = f32in
    q["f32_q3"] = Q1.quantize(f32in)
    q["blk88"] = d["dct_u8"][5]
    q["blk88_q"] = Q1.quantize(q["blk88"])                       # -> (1,1,3,8,8)
    q["blk388"] = DCT.transform(img3[:8, :8, :].transpose(2, 0, 1).astype(np.float32))
    q["blk388_q"] = Q1.quantize(q["blk388"])
    # E3-1_claude.py path: float32 block-of-3 quantised with a float32 DCT
    q["ties_in"] = (np.arange(-64, 64, dtype=np.float64).reshape(2, 1, 1, 8, 8) * 8.0)
    q["ties_q"] = Q1.quantize(q["ties_in"])
    np.savez_compressed(os.path.join(OUT, "quant.npz"), **q)

    # ---------------------------------------------------------------- zig-zag
    z = {}
    Z = sh_m.ZigZag()
    z["x5"] = rng.integers(-500, 500, (3, 2, 3, 8, 8)).astype(np.int32)
    z["flat"] = _quiet(Z.flatten, z["x5"])
    z["unflat"] = _quiet(Z.unflatten, z["flat"])
    z["x5_f64"] = rng.normal(size=(2, 2, 1, 8, 8))
    z["flat_f64"] = _quiet(Z.flatten, z["x5_f64"])
    z["x5_i16"] = rng.integers(-500, 500, (2, 2, 1, 8, 8)).astype(np.int16)
    z["flat_i16"] = _quiet(Z.flatten, z["x5_i16"])
    z["blk"] = rng.integers(0, 1000, (8, 8))
    z["scan"] = zz_m.zigzag_scan(z["blk"])
    z["order"] = Z.zigzag_order
    np.savez_compressed(os.path.join(OUT, "zigzag.npz"), **z)

    # ---------------------------------------------------------------- motion
    m = {}

    def me(name, ref, cur, sr):
        M = mo_m.MotionCompensator(search_range=sr)
        m[f"{name}_ref"], m[f"{name}_cur"] = ref, cur
        m[f"{name}_sr"] = np.array(sr)
        m[f"{name}_mv"] = M.compute_motion_vector(ref, cur)

    base = image_u8(rng, 96, 96, 1)[..., 0]
    shifted = np.roll(base, (3, -2), axis=(0, 1))
    me("shift_f64_sr4", base[:64, :64].astype(np.float64), shifted[:64, :64].astype(np.float64), 4)
    me("shift_f64_sr16", base[:64, :80].astype(np.float64), shifted[:64, :80].astype(np.float64), 16)
    me("flat_sr4", np.zeros((16, 16)), np.zeros((16, 16)), 4)
    nz = rng.normal(128, 40, (96, 80))
    me("nonint_f64_sr4", nz, np.roll(nz, (1, 2), axis=(0, 1)) + rng.normal(0, 0.3, (96, 80)), 4)
    me("f32_sr4", nz.astype(np.float32)[:64, :64],
       (np.roll(nz, (-2, 1), axis=(0, 1)) + rng.normal(0, 0.3, (96, 80))).astype(np.float32)[:64, :64], 4)
    me("u8mod_sr4", base[:64, :64], shifted[:64, :64], 4)
    me("u8mod_sr7", base[:48, :56], np.roll(base, (5, 4), axis=(0, 1))[:48, :56], 7)
    me("i16_sr4", (base[:48, :48].astype(np.int16) * 97), (shifted[:48, :48].astype(np.int16) * 89), 4)
    me("i32_sr3", base[:40, :40].astype(np.int32) * 1000003, shifted[:40, :40].astype(np.int32) * 999983, 3)
    # order-adversarial: 8-periodic reference -> every candidate window holds the same
    # multiset of values, so the winner is decided by the rounding of the summation order
    vals = np.array([0.1, 0.3, 0.7, 1.1, 1.3, 1.7, 2.9, 3.1])
    pat = vals[rng.integers(0, 8, (8, 8))]
    per = np.tile(pat, (6, 6))
    me("periodic_f64_sr8", per, np.full((48, 48), 0.05), 8)
    me("periodic_f32_sr8", per.astype(np.float32), np.full((48, 48), 0.05, np.float32), 8)
    me("periodic2_f64_sr5", per[:40, :40] * 1.7, np.full((40, 40), 0.3), 5)
    # motion compensation (including decoded indices that point out of the frame)
    M4 = mo_m.MotionCompensator(search_range=4)
    mv = m["shift_f64_sr4_mv"].copy()
    mv[0, 0, 0] = 0
    mv[-1, -1, 0] = 80
    m["mc_mv"] = mv
    m["mc_ref1"] = base[:64, :64, None].astype(np.float64)
    m["mc_out1"] = M4.reconstruct_with_motion_vector(m["mc_ref1"], mv)
    m["mc_ref3"] = image_u8(rng, 64, 64, 3)
    m["mc_out3"] = M4.reconstruct_with_motion_vector(m["mc_ref3"], mv)
    np.savez_compressed(os.path.join(OUT, "motion.npz"), **m)

    # ---------------------------------------------------------------- fused intra chain
    p = {}
    Q = pq_m.PatchQuant(quantization_scale=0.5)
    for C in (1, 3):
        img = image_u8(rng, 48, 64, C)
        blocks = DCT.transform(P.patch(img))
        qq = Q.quantize(blocks)
        p[f"img{C}"] = img
        p[f"q{C}"] = qq
        p[f"zz{C}"] = _quiet(sh_m.ZigZag().flatten, qq)
        p[f"rec{C}"] = DCT.inverse_transform(Q.dequantize(_quiet(sh_m.ZigZag().unflatten, p[f"zz{C}"])))
    np.savez_compressed(os.path.join(OUT, "intra.npz"), **p)
    make_zerorun(p)
    make_color()
    make_ch3()
    make_stats()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


def make_zerorun(intra):
    """ZeroRunCoder fixtures: encode streams of real zig-zag output and of adversarial
    sparse blocks, decode round trips, and the decoder's error cases (type + message)."""
    zr_m = _load("ivclab/entropy/zerorun.py", "ref_zerorun")
    rng = np.random.default_rng(40)
    z = {}

    def enc(name, x, eob=4000, bs=64):
        Z = zr_m.ZeroRunCoder(end_of_block=eob, block_size=bs)
        z[f"{name}_x"] = x
        z[f"{name}_eob"] = np.array(eob)
        z[f"{name}_bs"] = np.array(bs)
        z[f"{name}_sym"] = _quiet(Z.encode, x)

    enc("zz1", intra["zz1"])
    enc("zz3", intra["zz3"])
    sp = rng.integers(-40, 41, (6, 7, 3, 64)).astype(np.int32)
    sp[rng.random(sp.shape) < 0.8] = 0
    sp[0, 0, 0] = 0                                   # all-zero block
    sp[0, 0, 1] = 0
    sp[0, 0, 1, 63] = -7                              # only the last coefficient
    sp[0, 1, 0] = 0
    sp[0, 1, 0, 0] = 3                                # only the first
    sp[0, 1, 1] = np.where(np.arange(64) % 2 == 0, 1, 0)  # alternating
    sp[0, 1, 2] = rng.integers(1, 9, 64)              # no zeros
    sp[0, 2, 0] = 0
    sp[0, 2, 0, [5, 40]] = [4000, -4000]              # a value equal to EOB
    enc("sparse", sp)
    enc("eob1000", sp[:2], eob=1000)
    small = rng.integers(-3, 4, (4, 5, 1, 16)).astype(np.int32)
    small[rng.random(small.shape) < 0.5] = 0
    enc("bs16", small, bs=16)
    # decode: round trips, then the error paths of zerorun.py:46-88
    Z = zr_m.ZeroRunCoder()
    z["dec_sparse"] = _quiet(Z.decode, z["sparse_sym"], sp.shape[:3])
    z["dec_zz3"] = _quiet(Z.decode, z["zz3_sym"], intra["zz3"].shape[:3])
    good = z["sparse_sym"]
    cases = {
        "truncated": (good[:-5], sp.shape[:3]),
        "trailing_zero": (np.concatenate([good[:1], [0]]).astype(np.int32), (1, 1, 1)),
        "truncated_mid": (np.array([1, 2, 0, 3], np.int32), (1, 1, 1)),
        "ends_after_zero": (np.array([5, 0], np.int32), (1, 1, 1)),
        "ends_after_zero2": (np.array([4000, 7, 0], np.int32), (1, 1, 2)),
        "overflow": (np.array([0, 60, 1, 2, 3, 4, 5, 4000], np.int32), (1, 1, 1)),
        "overflow_run": (np.array([1, 0, 70, 4000], np.int32), (1, 1, 1)),
        "too_few": (np.array([1, 4000, 2, 4000], np.int32), (1, 1, 3)),
        "extra_ignored": (np.concatenate([good, [5, 6, 0]]).astype(np.int32), sp.shape[:3]),
        "negative_run": (np.array([0, -3, 5, 4000, 4000], np.int32), (1, 2, 1)),
        "early_eob_value": (np.array([7, 4000, 9, 4000], np.int32), (1, 1, 2)),
        "empty": (np.zeros(0, np.int32), (1, 1, 1)),
        "zero_blocks": (np.zeros(0, np.int32), (0, 1, 1)),
    }
    for k, (sym, shape) in cases.items():
        z[f"err_{k}_sym"] = sym
        z[f"err_{k}_shape"] = np.array(shape)
        try:
            z[f"err_{k}_out"] = _quiet(Z.decode, sym, shape)
            z[f"err_{k}_exc"] = np.array("")
        except Exception as e:  # noqa: BLE001  (the reference's exception is the fixture)
            z[f"err_{k}_exc"] = np.array(f"{type(e).__name__}: {e}")
    np.savez_compressed(os.path.join(OUT, "zerorun.npz"), **z)


def make_color():
    """Colour conversion fixtures (rgb2ycbcr goes through NumPy's matmul -> OpenBLAS: the
    fixtures record this container's NumPy 2.2 / OpenBLAS 0.3.29 results)."""
    co = _load("ivclab/signal/color.py", "ref_color")
    rng = np.random.default_rng(60)
    c = {}
    c["rgb_u8"] = rng.integers(0, 256, (48, 64, 3)).astype(np.uint8)
    c["rgb_u8_ycc"] = co.rgb2ycbcr(c["rgb_u8"])
    c["rgb_u8_gray"] = co.rgb2gray(c["rgb_u8"])
    c["rgb_f64"] = rng.normal(128, 60, (40, 32, 3))
    c["rgb_f64_ycc"] = co.rgb2ycbcr(c["rgb_f64"])
    c["rgb_f64_gray"] = co.rgb2gray(c["rgb_f64"])
    c["rgb_f32"] = rng.normal(128, 60, (16, 24, 3)).astype(np.float32)
    c["rgb_f32_ycc"] = co.rgb2ycbcr(c["rgb_f32"])
    c["rgb_f32_gray"] = co.rgb2gray(c["rgb_f32"])
    c["rgb_i16"] = rng.integers(-300, 300, (8, 8, 3)).astype(np.int16)
    c["rgb_i16_ycc"] = co.rgb2ycbcr(c["rgb_i16"])
    c["ycc_f64"] = rng.normal(128, 90, (40, 48, 3))             # includes values that clip
    c["ycc_f64_rgb"] = co.ycbcr2rgb(c["ycc_f64"])
    c["ycc_f32"] = rng.normal(128, 90, (16, 16, 3)).astype(np.float32)
    c["ycc_f32_rgb"] = co.ycbcr2rgb(c["ycc_f32"])
    c["ycc_u8"] = rng.integers(0, 256, (8, 16, 3)).astype(np.uint8)
    c["ycc_u8_rgb"] = co.ycbcr2rgb(c["ycc_u8"])
    c["ycc4_f64"] = rng.normal(128, 40, (8, 8, 4))              # a 4th channel is ignored
    c["ycc4_f64_rgb"] = co.ycbcr2rgb(c["ycc4_f64"])
    c["round_trip"] = co.ycbcr2rgb(co.rgb2ycbcr(c["rgb_u8"]))
    np.savez_compressed(os.path.join(OUT, "color.npz"), **c)


def satpic_standin(rng, H=256, W=256):
    """A synthetic 'satellite picture' (RGB uint8): smooth terrain-like fields per channel at
    two scales, field-boundary edges, and sensor noise."""
    def smooth(n):
        lo = rng.normal(0, 1, (H // n + 2, W // n + 2))
        return np.kron(lo, np.ones((n, n)))[:H, :W]
    y = 110 + 45 * smooth(32) + 20 * smooth(8)
    fields = (smooth(16) > 0.3) * 35
    img = np.stack([y + fields + 10 * smooth(4) * c for c in (0.8, 1.0, 0.6)], axis=-1)
    img += rng.normal(0, 6, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def make_ch3():
    """tests/ch3.py:18-47 on a committed synthetic stand-in for data/satpic1.bmp: the BMP
    (read back through PIL exactly as ivclab.utils.imread does, io.py:5-8) and the quantities
    the reference's own modules compute for each assertion."""
    from PIL import Image
    dct_m = _load("ivclab/signal/dct.py", "ref_dct")
    pq_m = _load("ivclab/quantization/patchquant.py", "ref_patchquant")
    sh_m = _load("ivclab/utils/shape.py", "ref_shape")
    me_m = _load("ivclab/utils/metrics.py", "ref_metrics")
    img = satpic_standin(np.random.default_rng(31415))
    path = os.path.join(OUT, "satpic_standin.bmp")
    Image.fromarray(img).save(path)
    with Image.open(path) as data:
        orig = np.asarray(data)
    assert np.array_equal(orig, img)
    P = sh_m.Patcher(window_size=(8, 8))
    D = dct_m.DiscreteCosineTransform(norm="ortho")
    Q = pq_m.PatchQuant(quantization_scale=1.0)
    patched = P.patch(orig)
    transformed = D.transform(patched)
    quantized = Q.quantize(patched)
    rec = P.unpatch(Q.dequantize(quantized))
    c = {"mean_energy": np.float64(np.mean(transformed ** 2)),
         "inverse_allclose": np.bool_(np.allclose(D.inverse_transform(transformed), patched)),
         "mean_q2": np.float64(np.mean(quantized ** 2)),
         "mse": np.float64(me_m.calc_mse(orig, rec)),
         "psnr": np.float64(me_m.calc_psnr(orig, rec))}
    np.savez_compressed(os.path.join(OUT, "ch3.npz"), **c)
    print({k: float(v) for k, v in c.items()})


def _load_package_module(dotted):
    """Import ivclab.<...> with the reference's package __init__ files of `ivclab` and
    `ivclab.entropy` bypassed (they pull in huffman.py -> the absent `constriction` wheel);
    every other module, __init__ included, runs as in the reference."""
    import types
    os.environ.setdefault("MPLBACKEND", "Agg")
    for pkg in ("ivclab", "ivclab.entropy"):
        if pkg not in sys.modules:
            m = types.ModuleType(pkg)
            m.__path__ = [os.path.join(REF, *pkg.split("."))]
            sys.modules[pkg] = m
    return importlib.import_module(dotted)


def make_stats():
    """stats_marg / smooth_pmf / calc_entropy fixtures (ivclab/entropy/entropy.py:6-51):
    integer images over unit edges, non-integer float images over float / non-uniform edges,
    an int bin count, NaN and +-inf samples, values on the closing edge."""
    en = _load_package_module("ivclab.entropy.entropy")
    rng = np.random.default_rng(77)
    s = {}
    cases = {
        "u8_full": (rng.integers(0, 256, (40, 50, 3)).astype(np.uint8), np.arange(256)),
        "i16_window": (rng.integers(-300, 300, (60, 70)).astype(np.int16), np.arange(-20, 41)),
        "i64_unit": (rng.integers(-(1 << 40), 1 << 40, 500).astype(np.int64), np.arange(-5, 6)),
        "f64_linspace": (rng.normal(128, 50, (64, 64)), np.linspace(0, 255, 52)),
        "f32_nonuniform": (rng.normal(0, 3, (30, 40)).astype(np.float32),
                           np.array([-9.0, -2.5, -1.0, -0.25, 0.0, 0.1, 1.0, 4.0, 9.5])),
        "f64_intbins": (rng.normal(10, 2, 777), 17),
        "f64_edges_special": (np.array([np.nan, 1.0, 2.0, 5.0, -np.inf, np.inf, 0.0, 4.999]),
                              np.array([0.0, 1.0, 2.0, 5.0])),
        "f64_inf_edges": (np.array([np.nan, 1.0, -np.inf, np.inf, 0.0]),
                          np.array([-np.inf, 0.0, np.inf])),
        "u8_float_edges": (rng.integers(0, 256, (32, 32)).astype(np.uint8), np.arange(0, 257, 4.0)),
        "u8_step_edges": (rng.integers(0, 256, (32, 32)).astype(np.uint8), np.arange(0, 256, 3)),
    }
    for k, (x, bins) in cases.items():
        s[f"{k}_x"] = x
        s[f"{k}_bins"] = np.asarray(bins)
        pmf = en.stats_marg(x, bins)
        s[f"{k}_pmf"] = pmf
        s[f"{k}_smooth"] = en.smooth_pmf(pmf)
        s[f"{k}_entropy"] = np.float64(en.calc_entropy(pmf))
    np.savez_compressed(os.path.join(OUT, "stats.npz"), **s)


if __name__ == "__main__":
    parts = sys.argv[1:]
    if not parts:
        sys.exit(main())
    for part in parts:
        {"ch3": make_ch3, "stats": make_stats}[part]()
