"""Where the class-API time goes: the 4K-luma and cfg2 chains
DCT.transform(Patcher.patch(img)) -> PatchQuant.quantize -> ZigZag.flatten timed call by call,
the host pieces alone (patch view, the contiguous gather, pinned-pool allocation of each
result), the raw PCIe rates of pinned copies (H2D, D2H, both at once), and the per-call
latency of the reference's per-block loop calls (exercises/ch3/E3-1_claude.py:47-60:
transform of one (8, 8) block, quantize of a (3, 8, 8) stack) against the oracle's.
    python tools/class_api_breakdown.py [--json out.json]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ivclab_amd import DiscreteCosineTransform, Patcher, PatchQuant, ZigZag  # noqa: E402
from ivclab_amd import _native as N  # noqa: E402


def tmin(fn, reps=7):
    fn()
    best = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best.append(time.perf_counter() - t0)
    return round(float(np.median(best)) * 1e3, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    dct, pq, zz, pt = DiscreteCosineTransform(), PatchQuant(1.0), ZigZag(), Patcher()
    rng = np.random.default_rng(1)
    cases = {"4k_luma": bench.intra_frames(1, 2160, 3840, seed=3, dev=dev)[0].cpu().numpy()[..., None],
             "cfg2_1080p_rgb": rng.integers(0, 256, (1080, 1920, 3), dtype=np.uint8)}
    out = {}
    for name, img in cases.items():
        p = pt.patch(img)
        d = dct.transform(p)
        q = pq.quantize(d)
        z = zz.flatten(q)
        r = {"bytes": {"image": img.nbytes, "dct_out": d.nbytes, "quant_out": q.nbytes,
                       "zigzag_out": z.nbytes}}
        r["patch_view_ms"] = tmin(lambda: pt.patch(img))
        r["gather_ms"] = tmin(lambda: np.ascontiguousarray(pt.patch(img)))
        r["dct_ms"] = tmin(lambda: dct.transform(p))
        r["quantize_ms"] = tmin(lambda: pq.quantize(d))
        r["zigzag_ms"] = tmin(lambda: zz.flatten(q))
        r["chain_ms"] = tmin(lambda: zz.flatten(pq.quantize(dct.transform(pt.patch(img)))))
        # the same without the host pipeline (every call in one piece), same process
        L = N.lib()
        N.check(L.ivc_set_host_pipeline(0))
        r["dct_nopipe_ms"] = tmin(lambda: dct.transform(p))
        r["quantize_nopipe_ms"] = tmin(lambda: pq.quantize(d))
        r["zigzag_nopipe_ms"] = tmin(lambda: zz.flatten(q))
        r["chain_nopipe_ms"] = tmin(lambda: zz.flatten(pq.quantize(dct.transform(pt.patch(img)))))
        N.check(L.ivc_set_host_pipeline(0))
        r["chain_again_ms"] = tmin(lambda: zz.flatten(pq.quantize(dct.transform(pt.patch(img)))))
        want = zz.flatten(pq.quantize(dct.transform(np.ascontiguousarray(p))))
        assert np.array_equal(zz.flatten(pq.quantize(dct.transform(pt.patch(img)))), want)
        for k, a in (("dct_out", d), ("quant_out", q), ("zigzag_out", z)):
            r[f"alloc_{k}_ms"] = tmin(lambda: N.empty(a.shape, a.dtype))
        out[name] = r
        print(name, json.dumps(r), flush=True)
    # raw pinned PCIe rates (torch, 64 MiB)
    n = 64 << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    g = torch.empty(n, dtype=torch.uint8, device=dev)
    g2 = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        g.copy_(h, non_blocking=True)
        torch.cuda.synchronize()

    def d2h():
        h.copy_(g, non_blocking=True)
        torch.cuda.synchronize()

    def both():
        with torch.cuda.stream(s1):
            g.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(g2, non_blocking=True)
        torch.cuda.synchronize()

    pc = {"h2d_GBs": round(n / tmin(h2d) / 1e6, 1), "d2h_GBs": round(n / tmin(d2h) / 1e6, 1),
          "both_GBs_each": round(n / tmin(both) / 1e6, 1)}
    out["pcie"] = pc
    print("pcie", json.dumps(pc), flush=True)
    # small calls: one (8, 8) block through transform, one (3, 8, 8) stack through quantize
    from oracle import ivc_oracle as O
    blk = rng.integers(0, 256, (8, 8)).astype(np.float64)
    stk = rng.normal(0, 50, (3, 8, 8))
    reps = 200

    def per_call(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return round((time.perf_counter() - t0) / reps * 1e6, 2)

    sc = {"transform_8x8_us": per_call(lambda: dct.transform(blk)),
          "transform_8x8_oracle_us": per_call(lambda: O.dct_transform(blk)),
          "quantize_3x8x8_us": per_call(lambda: pq.quantize(stk)),
          "quantize_3x8x8_oracle_us": per_call(lambda: O.quantize(stk, 1.0))}
    assert np.array_equal(dct.transform(blk).view(np.uint64), O.dct_transform(blk).view(np.uint64))
    assert np.array_equal(pq.quantize(stk), O.quantize(stk, 1.0))
    out["small_call"] = sc
    print("small_call", json.dumps(sc), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
