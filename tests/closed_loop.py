"""Test-side restatement of the closed-loop P-frame codec of the reference's chapter-4
exercise (exercises/ch4/ex1.py:9-373, `SimpleVideoCodec.encode_decode`, driven as in its
__main__ loop :385-410) — the reference's only working P-frame path (VideoCodec itself
raises).  Written from the exercise's behaviour, not copied; it keeps exactly the data flow
that decides the reconstruction:

  frame 0 (I):  YCbCr of the float32 RGB frame (:178); Y coded by IntraCodec
                (train_huffman_from_image + encode_decode, :194-201, plane 0 of the
                3-plane reconstruction); Cb and Cr passed through uncoded (:202-203)
  frame n (P):  ME on the DECODER's previous luma reconstruction (:228, float64 NumPy
                semantics), MC of Y, Cb and Cr with the luma vectors (:270-279), luma
                residual through a second IntraCodec (:333-342), reconstruction
                prediction + decoded residual for Y, the predictions for Cb/Cr (:345-349)
  output:       clip to [0, 255], ycbcr2rgb, astype(uint8) (:361-370)

and the rate bookkeeping in simplified form: every frame's symbols (I-frame luma, P-frame
motion indices and luma residual) are Huffman-coded with a coder trained on their own
non-zero histogram (the exercise's `_adaptive_encode_symbols`, :41-77).  The exercise's
trained-on-frame-1 coders with nearest-symbol remapping only change bit counts; bit counts
are checked against entropy bounds, not pinned (constriction is absent).

`api` supplies the primitives: the drop-in (`ivclab.*` names under install_as_ivclab, on the
GPU) or the oracle (oracle/ivc_oracle.py on the CPU, bits skipped).
"""
from __future__ import annotations

import numpy as np


def adaptive_bits(api, symbols):
    """ex1.py:41-77: histogram over [min, max + 1] by stats_marg, non-zero bins compacted,
    a fresh Huffman coder trained on them, bits of the compacted message."""
    s = np.asarray(symbols)
    lo, hi = int(s.min()), int(s.max())
    edges = np.arange(lo, hi + 2)
    hist = api.stats_marg(s, pixel_range=edges)
    keep = hist > 0
    index = np.cumsum(keep) - 1                       # compact index of every kept bin
    compact = index[s.astype(np.int64) - lo]
    coder = api.HuffmanCoder()
    coder.train(hist[keep])
    _, bits = coder.encode(compact)
    return float(bits), hist[keep], int(s.size)


def run(api, frames_rgb, q_scale, sr):
    """Encode/decode the sequence; returns per-frame dicts with the RGB reconstruction, the
    decoder's float64 YCbCr state, motion vectors (None for the I-frame) and bit records."""
    intra = api.IntraCodec(quantization_scale=q_scale, bounds=(-1000, 4000), end_of_block=4000,
                           block_shape=(8, 8))
    resid_codec = api.IntraCodec(quantization_scale=q_scale, bounds=(-1000, 4000),
                                 end_of_block=4000, block_shape=(8, 8))
    mc = api.MotionCompensator(search_range=sr)
    state = None
    out = []
    for n, frame in enumerate(frames_rgb):
        ycc = api.rgb2ycbcr(frame.astype(np.float32))
        y, cb, cr = ycc[..., 0], ycc[..., 1], ycc[..., 2]
        rec = {"bits": []}
        if n == 0:
            if api.bits:
                rec["bits"].append(adaptive_bits(api, intra.image2symbols(y, is_source_rgb=False)))
            intra.train_huffman_from_image(y, is_source_rgb=False)
            ry = intra.encode_decode(y, is_source_rgb=False)[0]
            ry = ry[..., 0] if ry.ndim == 3 else ry
            rcb, rcr = cb, cr
            mv = None
        else:
            dy, dcb, dcr = state[..., 0], state[..., 1], state[..., 2]
            mv = mc.compute_motion_vector(dy, y)
            py = mc.reconstruct_with_motion_vector(dy[..., None], mv)[..., 0]
            pcb = mc.reconstruct_with_motion_vector(dcb[..., None], mv)[..., 0]
            pcr = mc.reconstruct_with_motion_vector(dcr[..., None], mv)[..., 0]
            res = y - py
            if api.bits:
                rec["bits"].append(adaptive_bits(api, mv.flatten()))
                rec["bits"].append(adaptive_bits(api, resid_codec.image2symbols(res, is_source_rgb=False)))
            resid_codec.train_huffman_from_image(res, is_source_rgb=False)
            rr = resid_codec.encode_decode(res, is_source_rgb=False)[0]
            rr = rr[..., 0] if rr.ndim == 3 else rr
            ry, rcb, rcr = py + rr, pcb, pcr
        state = np.stack([np.asarray(ry).reshape(cb.shape), rcb, rcr], axis=-1)
        disp = ycc.copy()
        disp[..., 0] = np.clip(state[..., 0], 0, 255)
        disp[..., 1] = np.clip(state[..., 1], 0, 255)
        disp[..., 2] = np.clip(state[..., 2], 0, 255)
        rec["rgb"] = api.ycbcr2rgb(disp).astype(np.uint8)
        rec["state"] = state
        rec["mv"] = mv
        out.append(rec)
    return out


def synthetic_sequence(F=8, H=64, W=80, seed=7):
    """An RGB sequence with global motion inside +-4 (the exercise's search range) over a
    smooth texture plus noise, one flat region (ME tie-break) and a scene cut-free drift."""
    rng = np.random.default_rng(seed)
    P = 8
    yy, xx = np.mgrid[0:H + 2 * P, 0:W + 2 * P]
    base = np.stack([128 + 70 * np.sin(xx / (9.0 + 2 * c)) * np.cos(yy / (7.0 + c)) + 0.4 * (xx - yy)
                     for c in range(3)], axis=-1)
    base = base + rng.normal(0, 5, base.shape)
    frames = []
    for f in range(F):
        dy, dx = (f % 5) - 2, (3 * f % 7) - 3
        fr = base[P + dy:P + dy + H, P + dx:P + dx + W] + rng.normal(0, 2, (H, W, 3))
        fr[8:24, 40:64] = 90 + 10 * (f % 2)                 # flat patch
        frames.append(np.clip(fr, 0, 255).astype(np.uint8))
    return np.stack(frames)
