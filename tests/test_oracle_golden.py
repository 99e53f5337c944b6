"""Pin the CPU oracle (oracle/ivc_oracle.py) against the golden vectors the reference itself
produced (tests/golden/make_golden.py).  Bit-exact comparisons throughout."""
import numpy as np
import pytest

from oracle import ivc_oracle as O


def bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def test_dct_golden(golden):
    d = golden("dct")
    assert bits_equal(O.dct_transform(d["x_u8"]), d["dct_u8"])
    assert bits_equal(O.dct_transform(d["x_f64"]), d["dct_f64"])
    assert bits_equal(O.dct_inverse(d["x_f64"]), d["idct_f64"])
    assert bits_equal(O.dct_transform(d["x_f32"]), d["dct_f32"])
    assert bits_equal(O.dct_inverse(d["x_f32"]), d["idct_f32"])
    assert bits_equal(O.dct_inverse(d["x_i32"]), d["idct_i32"])
    assert bits_equal(O.dct_transform(d["x_i16"]), d["dct_i16"])
    for norm in ("backward", "forward"):
        assert bits_equal(O.dct_transform(d["x_f64"][:64], norm), d[f"dct_f64_{norm}"])
        assert bits_equal(O.dct_inverse(d["x_f64"][:64], norm), d[f"idct_f64_{norm}"])
    assert bits_equal(O.dct_transform(O.patch(d["x_img"])), d["dct_img"])


def test_quant_golden(golden):
    q = golden("quant")
    d1 = O.dct_transform(O.patch(q["img1"]))
    d3 = O.dct_transform(O.patch(q["img3"]))
    for i, s in enumerate(q["scales"]):
        s = float(s)
        assert bits_equal(O.quant_table(s), q[f"table_{i}"])
        assert bits_equal(O.quantize(d1, s), q[f"q1_{i}"])
        assert bits_equal(O.quantize(d3, s), q[f"q3_{i}"])
        assert bits_equal(O.dequantize(q[f"q1_{i}"], s), q[f"dq1_{i}"])
        assert bits_equal(O.dequantize(q[f"q3_{i}"], s), q[f"dq3_{i}"])
        assert bits_equal(O.dct_inverse(q[f"dq3_{i}"]), q[f"idq3_{i}"])
    assert bits_equal(O.quantize(O.patch(q["img3"])), q["raw_q3"])
    assert bits_equal(O.dequantize(q["raw_q3"]), q["raw_dq3"])
    assert bits_equal(O.quantize(q["f32_dct3"]), q["f32_q3"])
    assert bits_equal(O.quantize(q["blk88"]), q["blk88_q"])
    assert O.quantize(q["blk88"]).shape == (1, 1, 3, 8, 8)
    assert bits_equal(O.quantize(q["blk388"]), q["blk388_q"])
    assert bits_equal(O.quantize(q["ties_in"]), q["ties_q"])


def test_zigzag_golden(golden):
    z = golden("zigzag")
    assert np.array_equal(z["order"], O.ZZ_ORDER)
    assert bits_equal(O.zigzag_flatten(z["x5"]), z["flat"])
    assert bits_equal(O.zigzag_unflatten(z["flat"]), z["unflat"])
    assert bits_equal(O.zigzag_flatten(z["x5_f64"]), z["flat_f64"])
    assert bits_equal(O.zigzag_flatten(z["x5_i16"]), z["flat_i16"])
    assert bits_equal(O.zigzag_scan(z["blk"]), z["scan"])


ME_CASES = ["shift_f64_sr4", "shift_f64_sr16", "flat_sr4", "nonint_f64_sr4", "f32_sr4",
            "u8mod_sr4", "u8mod_sr7", "i16_sr4", "i32_sr3", "periodic_f64_sr8",
            "periodic_f32_sr8", "periodic2_f64_sr5"]


@pytest.mark.parametrize("case", ME_CASES)
def test_motion_golden(golden, case):
    m = golden("motion")
    ref, cur, sr = m[f"{case}_ref"], m[f"{case}_cur"], int(m[f"{case}_sr"])
    assert bits_equal(O.motion_vectors(ref, cur, sr), m[f"{case}_mv"])
    if ref.size <= 64 * 64 and sr <= 4:
        assert bits_equal(O.motion_vectors_loop(ref, cur, sr), m[f"{case}_mv"])


def test_motion_flat_tiebreak(golden):
    m = golden("motion")
    assert m["flat_sr4_mv"][..., 0].tolist() == [[40, 36], [4, 0]]


def test_mc_golden(golden):
    m = golden("motion")
    assert bits_equal(O.motion_compensate(m["mc_ref1"], m["mc_mv"], 4), m["mc_out1"])
    assert bits_equal(O.motion_compensate(m["mc_ref3"], m["mc_mv"], 4), m["mc_out3"])


def test_intra_golden(golden):
    p = golden("intra")
    for C in (1, 3):
        assert bits_equal(O.intra_encode(p[f"img{C}"], 0.5), p[f"q{C}"])
        assert bits_equal(O.intra_encode(p[f"img{C}"], 0.5, zigzag=True), p[f"zz{C}"])
        assert bits_equal(O.intra_decode(p[f"zz{C}"], 0.5, unzigzag=True), p[f"rec{C}"])


@pytest.mark.parametrize("case", ME_CASES)
def test_c_oracle_motion_golden(golden, case):
    from oracle import c_motion_vectors
    m = golden("motion")
    ref, cur, sr = m[f"{case}_ref"], m[f"{case}_cur"], int(m[f"{case}_sr"])
    cur = cur.astype(np.result_type(ref.dtype, cur.dtype))
    ref = ref.astype(cur.dtype)
    assert bits_equal(c_motion_vectors(ref, cur, sr).astype(int), m[f"{case}_mv"])


def test_c_oracle_exact_u8_equals_f64(golden):
    from oracle import c_motion_vectors
    rng = np.random.default_rng(7)
    a = rng.integers(0, 256, (64, 72), dtype=np.uint8)
    b = np.roll(a, (2, -3), axis=(0, 1))
    b[::5] = rng.integers(0, 256, b[::5].shape)
    ref = O.motion_vectors(a.astype(np.float64), b.astype(np.float64), 6)
    assert np.array_equal(c_motion_vectors(a, b, 6, exact_u8=True), ref)
    assert np.array_equal(c_motion_vectors(a, b, 6, rows=(2, 5)), O.motion_vectors(a, b, 6)[2:5])


def test_c_oracle_mc_golden(golden):
    from oracle import c_motion_compensate
    m = golden("motion")
    assert bits_equal(c_motion_compensate(m["mc_ref1"], m["mc_mv"], 4), m["mc_out1"])
    assert bits_equal(c_motion_compensate(m["mc_ref3"], m["mc_mv"], 4), m["mc_out3"])


ZR_ENC = ["zz1", "zz3", "sparse", "eob1000", "bs16"]
ZR_ERR = ["truncated", "trailing_zero", "truncated_mid", "ends_after_zero", "ends_after_zero2",
          "overflow", "overflow_run", "too_few", "extra_ignored", "negative_run",
          "early_eob_value", "empty"]


@pytest.mark.parametrize("case", ZR_ENC)
def test_zerorun_encode_golden(golden, case):
    z = golden("zerorun")
    x, eob, bs = z[f"{case}_x"], int(z[f"{case}_eob"]), int(z[f"{case}_bs"])
    assert bits_equal(O.zerorun_encode(x, eob, bs), z[f"{case}_sym"])
    assert bits_equal(O.zerorun_encode_fast(x, eob, bs), z[f"{case}_sym"])


def test_zerorun_decode_golden(golden):
    z = golden("zerorun")
    assert bits_equal(O.zerorun_decode(z["sparse_sym"], z["sparse_x"].shape[:3]), z["dec_sparse"])
    assert bits_equal(O.zerorun_decode(z["zz3_sym"], z["zz3_x"].shape[:3]), z["dec_zz3"])


@pytest.mark.parametrize("case", ZR_ERR)
def test_zerorun_decode_errors_golden(golden, case):
    """The decoder's outcome on malformed / edge streams, exception type and message
    included, as the reference produced it."""
    z = golden("zerorun")
    sym, shape, exc = z[f"err_{case}_sym"], tuple(int(v) for v in z[f"err_{case}_shape"]), str(z[f"err_{case}_exc"])
    if exc:
        with pytest.raises(Exception) as ei:
            O.zerorun_decode(sym, shape)
        assert f"{type(ei.value).__name__}: {ei.value}" == exc
    else:
        assert bits_equal(O.zerorun_decode(sym, shape), z[f"err_{case}_out"])


def test_color_golden(golden):
    c = golden("color")
    for k in ("rgb_u8", "rgb_f64", "rgb_f32", "rgb_i16"):
        assert bits_equal(O.rgb2ycbcr(c[k]), c[f"{k}_ycc"]), k
    for k in ("rgb_u8", "rgb_f64", "rgb_f32"):
        assert bits_equal(O.rgb2gray(c[k]), c[f"{k}_gray"]), k
    for k in ("ycc_f64", "ycc_f32", "ycc_u8", "ycc4_f64"):
        assert bits_equal(O.ycbcr2rgb(c[k]), c[f"{k}_rgb"]), k


def test_rgb2ycbcr_is_korder_fma(golden):
    """The kernel's arithmetic (k-order fused multiply-adds, then the offset) reproduces the
    reference's matmul on the fixtures — the claim ivc_color.hip rests on."""
    c = golden("color")
    for k in ("rgb_u8", "rgb_f64"):
        x = c[k][:6, :8]
        assert bits_equal(O.rgb2ycbcr_fma(x), c[f"{k}_ycc"][:6, :8]), k


STATS = ["u8_full", "i16_window", "i64_unit", "f64_linspace", "f32_nonuniform", "f64_intbins",
         "f64_edges_special", "f64_inf_edges", "u8_float_edges", "u8_step_edges"]


@pytest.mark.parametrize("case", STATS)
def test_stats_golden(golden, case):
    """stats_marg / smooth_pmf / calc_entropy (entropy.py:6-51) against the reference's own
    outputs: integer and float data, unit / float / non-uniform edges, an int bin count,
    NaN and infinities, values on the closing edge."""
    s = golden("stats")
    x, bins = s[f"{case}_x"], s[f"{case}_bins"]
    bins = int(bins) if bins.ndim == 0 else bins
    pmf = O.stats_marg(x, bins)
    assert bits_equal(pmf, s[f"{case}_pmf"])
    assert bits_equal(O.smooth_pmf(pmf), s[f"{case}_smooth"])
    assert bits_equal(np.float64(O.calc_entropy(pmf)), s[f"{case}_entropy"])


def test_c_inter_encode_matches_oracle_chain():
    """oracle.c_inter_encode (C ME + block copy + NumPy DCT/quant, row-restricted) equals
    ivc_oracle.inter_encode, whole frame and on block-row stripes."""
    from oracle import c_inter_encode
    rng = np.random.default_rng(11)
    a = rng.integers(0, 256, (48, 64), dtype=np.uint8)
    b = np.roll(a, (2, -3), (0, 1))
    b[5:20, 7:30] = rng.integers(0, 256, (15, 23))
    for zz in (False, True):
        mv, q = O.inter_encode(a, b, 4, 1.0, zz)
        mv2, q2 = c_inter_encode(a, b, 4, 1.0, zz)
        assert bits_equal(mv2, mv.astype(np.int64)) and bits_equal(q2, q)
        for rows in ((0, 2), (2, 5), (5, 6)):
            mv3, q3 = c_inter_encode(a, b, 4, 1.0, zz, rows=rows)
            assert bits_equal(mv3, mv[rows[0]:rows[1]].astype(np.int64))
            assert bits_equal(q3, q[rows[0]:rows[1]])
