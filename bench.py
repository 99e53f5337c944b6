"""Benchmark of the ivclab block-codec hot path on MI355X (contract: one JSON line on rank 0).

Headline (`value`, BASELINE.json configs[2], the metric's "4K intra DCT+quant" half): a batch
of 256 synthetic 3840x2160 luma frames per GPU, resident in HBM, through the fused
patch -> DCT-II -> quantise kernel (reference-equivalent output: [F,270,480,3,64] int32, the
C = 1 -> 3-plane broadcast of patchquant.py:59).  One step = one pass over the batch.
`roofline` prices that kernel against HBM (13 B/px algorithmic, HIP events on its stream;
`traffic` from the committed PMC record), `cpu_baseline` times the reference's algorithm
(oracle) on one host core, `cpu_baseline_multicore` on the box's cores.

Also reported from the same run:
  zerorun / image2symbols  ZeroRunCoder on the zig-zag output, and pixels -> symbols fused
  exchange                 global Huffman-table input: alphabet bounds (all-reduce) and the
                           symbol histogram (all-gather), as IntraCodec trains it
  inter                    configs[3]: 1080p x 300, +-16 full-search ME + MC + residual DCT+quant
  sharded                  configs[4]: 8K x 120 frames split across the ranks (strong scaling),
                           ME + residual DCT+quant + one histogram all-gather per step
Multi-GPU: one process per GPU (torch.distributed, RCCL); cfg3/cfg4 are weak-scaled (each
rank owns its frames), cfg5 strong-scaled.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--no-inter] [--no-cpu]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
INT_VALU_PEAK_TOPS = 78.6      # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz, 32-bit integer ops/s
HIST_LO, HIST_BINS = -4096, 8192


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        # rehearsal of the multi-rank path on a 1-GPU box: IVC_BENCH_BACKEND=gloo puts every
        # rank on cuda:0 (RCCL needs one GPU per rank); the driver's runs use nccl = RCCL
        backend = os.environ.get("IVC_BENCH_BACKEND", "nccl")
        dev = local if backend == "nccl" else local % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        return dist, rank, world, dev
    torch.cuda.set_device(0)
    return None, 0, 1, 0


def coll_name(dist):
    b = dist.get_backend()
    return "RCCL" if b == "nccl" else b


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, v):
    if dist is None:
        return v
    t = torch.tensor([v], dtype=torch.float64,
                     device="cpu" if dist.get_backend() == "gloo" else "cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---------------------------------------------------------------- synthetic frames ------
def intra_frames(F, H, W, seed, dev):
    """Per 8x8 block: ~50% uniform noise, 25% flat (DC ties), 25% ramps; seeded, on device."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    out = torch.empty((F, H, W), dtype=torch.uint8, device=dev)
    h, w = H // 8, W // 8
    ii = torch.arange(8, device=dev)
    ramp = (ii[:, None] + ii[None, :]).to(torch.int16)                     # [8, 8]
    for f in range(F):
        x = torch.randint(0, 256, (H, W), dtype=torch.uint8, device=dev, generator=g)
        kind = torch.randint(0, 4, (h, 1, w, 1), device=dev, generator=g)
        base = torch.randint(0, 256, (h, 1, w, 1), dtype=torch.int16, device=dev, generator=g)
        slope = torch.randint(1, 17, (h, 1, w, 1), dtype=torch.int16, device=dev, generator=g)
        xb = x.view(h, 8, w, 8)
        flat = base.expand(h, 8, w, 8).to(torch.uint8)
        rmp = (ramp.view(1, 8, 1, 8) * slope).clamp(0, 255).to(torch.uint8)
        xb = torch.where(kind == 0, flat, xb)
        xb = torch.where(kind == 1, rmp.expand(h, 8, w, 8), xb)
        out[f] = xb.reshape(H, W)
    return out


def inter_frames(F, H, W, seed, dev, first=0):
    """Frames first .. first+F-1 of a sequence: a smooth base texture shifted by
    (dy, dx) = ((f % 7) - 3, (2f % 9) - 4) plus +-2 noise, so consecutive
    frames differ by a motion within +-16.  Frame f depends only on (seed, f), so ranks
    generating disjoint frame ranges of one sequence agree on the shared halo frame."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    P = 16
    lo = torch.randint(0, 256, (1, 1, (H + 2 * P) // 4 + 2, (W + 2 * P) // 4 + 2),
                       device=dev, generator=g).float()
    base = torch.nn.functional.interpolate(lo, scale_factor=4, mode="bilinear", align_corners=False)
    base = base[0, 0, :H + 2 * P, :W + 2 * P]
    base = base + torch.randint(-12, 13, base.shape, device=dev, generator=g).float()
    out = torch.empty((F, H, W), dtype=torch.uint8, device=dev)
    for i in range(F):
        f = first + i
        gf = torch.Generator(device=dev)
        gf.manual_seed(seed * 1000003 + f)
        dy, dx = (f % 7) - 3, (2 * f % 9) - 4
        fr = base[P + dy:P + dy + H, P + dx:P + dx + W]
        fr = fr + torch.randint(-2, 3, (H, W), device=dev, generator=gf).float()
        out[i] = fr.round().clamp(0, 255).to(torch.uint8)
    return out


# ---------------------------------------------------------------- timing ----------------
def timed(dist, fn, steps, warmup):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize; returns
    (max-over-ranks wall seconds, per-step device-event ms of fn's kernels)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(dist)
    wall = max_over_ranks(dist, t1 - t0)
    return wall, ev0.elapsed_time(ev1) / steps


def cpu_baseline_intra(frames_host, budget_s=12.0):
    """Oracle (NumPy/SciPy restatement of the reference, single thread, as the reference
    runs) on whole 4K frames until ~budget_s of CPU work; returns Mpx/s and frames done."""
    from oracle import ivc_oracle as O
    n, t0 = 0, time.perf_counter()
    while n < len(frames_host):
        O.intra_encode(frames_host[n][..., None], 1.0)
        n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    H, W = frames_host[0].shape
    return n * H * W / dt / 1e6, n, dt


def cpu_baseline_me(frames_host, sr, budget_s=10.0):
    """The reference's literal ME loop (oracle motion_vectors_loop on float64 frames) on a
    stripe of block rows of one 1080p pair, extrapolated per valid candidate."""
    from oracle import ivc_oracle as O
    a = frames_host[0].astype(np.float64)
    b = frames_host[1].astype(np.float64)
    H, W = a.shape
    # a 32-row sub-frame from the middle of the pair (4 block rows x W)
    sub_h = 32
    y0 = (H // 2) // 8 * 8
    ra, rb = a[y0:y0 + sub_h], b[y0:y0 + sub_h]
    t0 = time.perf_counter()
    O.motion_vectors_loop(ra, rb, sr)
    dt = time.perf_counter() - t0
    n = 2 * sr + 1

    def valid_count(h, w):
        by = np.arange(h // 8) * 8
        bx = np.arange(w // 8) * 8
        d = np.arange(-sr, sr + 1)
        vy = ((by[:, None] + d[None]) >= 0) & ((by[:, None] + d[None] + 8) <= h)
        vx = ((bx[:, None] + d[None]) >= 0) & ((bx[:, None] + d[None] + 8) <= w)
        return int(vy.sum(1).sum() * vx.sum(1).sum())

    per_cand = dt / valid_count(sub_h, W)
    frame_s = per_cand * valid_count(H, W)
    return H * W / frame_s / 1e6, per_cand, n


def cpu_workers():
    """Host cores this process may use (the GPU box's share, not the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_pool(intra_host, me_pair, sr, budget_s=8.0):
    """The same oracle paths frame-sharded over the host cores (multiprocessing, spawn):
    intra on whole frames (each worker its own frames) and the ME loop on block-row
    stripes (each worker its own stripe).  Returns (intra Mpx/s, ME Mpx/s, workers)."""
    import multiprocessing as mp
    from oracle import cpu_pool
    P = cpu_workers()
    ctx = mp.get_context("spawn")
    with ctx.Pool(P) as pool:
        pool.map(cpu_pool.warm, range(P))
        # intra: 1 frame per worker per round until the budget is spent
        H, W = intra_host[0].shape
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget_s / 2:
            chunks = [[intra_host[(done + i) % len(intra_host)]] for i in range(P)]
            done += sum(pool.map(cpu_pool.intra_frames, chunks))
        intra_mpx = done * H * W / (time.perf_counter() - t0) / 1e6
        # ME: P stripes of 16 rows (2 block rows) from the middle of a 1080p pair
        a = me_pair[0].astype(np.float64)
        b = me_pair[1].astype(np.float64)
        Hm, Wm = a.shape
        y0 = (Hm // 2 - 8 * P) // 8 * 8
        stripes = [(a[y0 + 16 * i:y0 + 16 * i + 16], b[y0 + 16 * i:y0 + 16 * i + 16], sr)
                   for i in range(P)]
        t0 = time.perf_counter()
        pool.map(cpu_pool.me_stripe, stripes)
        dt = time.perf_counter() - t0
    # per-candidate rate of the stripes, extrapolated to whole frames like the 1-core leg
    n = 2 * sr + 1

    def valid(h, w):
        by, bx, d = np.arange(h // 8) * 8, np.arange(w // 8) * 8, np.arange(-sr, sr + 1)
        vy = ((by[:, None] + d[None]) >= 0) & ((by[:, None] + d[None] + 8) <= h)
        vx = ((bx[:, None] + d[None]) >= 0) & ((bx[:, None] + d[None] + 8) <= w)
        return int(vy.sum(1).sum() * vx.sum(1).sum())

    del n
    cand_rate = P * valid(16, Wm) / dt
    me_mpx = Hm * Wm / (valid(Hm, Wm) / cand_rate) / 1e6
    return intra_mpx, me_mpx, P


# ---------------------------------------------------------------- main ------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--inter-frames", type=int, default=300)
    ap.add_argument("--inter-steps", type=int, default=3)
    ap.add_argument("--sr", type=int, default=16)
    ap.add_argument("--zigzag", action="store_true")
    ap.add_argument("--no-inter", action="store_true")
    ap.add_argument("--no-intra", action="store_true", help="profiling aid: skip the cfg3 leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-sharded", action="store_true", help="skip the cfg5 8K leg")
    ap.add_argument("--no-cpu-pool", action="store_true", help="skip the multi-core CPU leg")
    ap.add_argument("--sharded-frames", type=int, default=120)
    ap.add_argument("--sharded-steps", type=int, default=3)
    ap.add_argument("--sharded-hist-wg", type=int, default=2,
                    help="workgroups per CU of the side-stream histograms in the cfg5 step")
    ap.add_argument("--sharded-chunk", type=int, default=8,
                    help="frame pairs per inter_encode call in the cfg5 step; the histogram of "
                         "chunk k runs on a side stream while chunk k+1 is encoded (0: one call)")
    args = ap.parse_args()

    dist, rank, world, local = dist_setup(args.gpus)
    dev = torch.device("cuda", torch.cuda.current_device())
    import ivclab_amd.device as D
    from ivclab_amd.distributed import global_bounds, global_histogram
    from ivclab_amd.entropy.stats import (entropy_bits, huffman_bounds, smooth_pmf,
                                          stats_marg_from_counts)
    from ivclab_amd import PatchQuant
    table = PatchQuant(1.0).get_quantization_table()

    # ---- cfg3: 4K intra DCT + quant -------------------------------------------------------
    F, H, W = args.frames, args.height, args.width
    if args.no_intra:
        F = 1
    frames = intra_frames(F, H, W, seed=3 + 1000 * rank, dev=dev).view(F, H, W, 1)
    out = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)

    def step():
        D.intra_encode(frames, table, out, zigzag=args.zigzag)

    wall, kern_ms = timed(dist, step, args.steps, args.warmup)
    from ivclab_amd import _native as N
    pace_rate, pace_late = N.lib().ivc_store_pace(), N.lib().ivc_store_pace_late()

    # write-stream ceiling for this buffer: the same 12 B/px of int32 output written by
    # torch's vectorised fill kernel (no reads) — what the store side alone can reach
    _, fill_ms = timed(None, lambda: out.fill_(0), 3, 1)
    fill_gbs = out.numel() * 4 / (fill_ms * 1e-3) / 1e9
    px_step = F * H * W
    value = world * px_step * args.steps / wall / 1e6
    algo_bytes = px_step * 13                        # 1 B u8 in + 3 x 4 B int32 out per px
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9

    # ---- symbols for the global Huffman table (IntraCodec.image2symbols + training input,
    # intracodec.py:32-90,149-166): the same frames with zig-zag, zero-run coded on the GPU;
    # global alphabet bounds (one all-reduce), per-rank histogram, one all-gather
    D.intra_encode(frames, table, out, zigzag=True)
    nblk = out.numel() // 64
    blocks = out.view(nblk, 64)
    offs = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
    probe = torch.empty(1, dtype=torch.int32, device=dev)
    D.zerorun_encode(blocks, offs, probe)
    nsym = int(offs[-1].item())
    sym = torch.empty(nsym, dtype=torch.int32, device=dev)
    zwall, zms = timed(dist, lambda: D.zerorun_encode(blocks, offs, sym), 3, 1)
    # the same stream straight from the pixels (fused: the coefficients never reach HBM)
    nsym_d = torch.zeros(1, dtype=torch.int64, device=dev)
    fwall, fms = timed(dist, lambda: D.intra_symbols(frames, table, sym, nsym_d), 3, 1)
    fused_same = bool(int(nsym_d.item()) == nsym)
    mm = torch.empty(2, dtype=torch.int32, device=dev)

    def exchange():
        D.minmax(sym, mm)
        lo, hi = global_bounds(mm)
        b0, b1 = huffman_bounds(lo, hi)
        hist = torch.zeros(b1 - b0 - 1, dtype=torch.int64, device=dev)
        D.histogram(sym, b0, hist)
        return b0, b1, global_histogram(hist)

    exchange()                      # warm-up: first-launch and allocator costs stay untimed
    torch.cuda.synchronize()
    barrier(dist)
    t_ex = time.perf_counter()
    b0, b1, ghist = exchange()
    torch.cuda.synchronize()
    exchange_ms = (time.perf_counter() - t_ex) * 1e3
    counts = ghist.cpu().numpy()
    total_syms = int(counts.sum())
    pmf = smooth_pmf(stats_marg_from_counts(counts))
    del sym, offs, blocks
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_intra_latest.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            rec = json.load(fh)
        if rec.get("frames") == F and rec.get("H") == H and rec.get("W") == W:
            traffic = rec.get("hbm_bytes_per_launch")

    result = {
        "metric": "Mpixels/s: 4K intra DCT+quant and ±16 full-search ME, 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded on-device 4K luma: 50% noise / 25% flat / 25% ramp blocks)",
        "config": {"workload": f"cfg3: {F} x {W}x{H} luma u8 per GPU, fused patch->DCT->quant "
                               f"(scale 1.0, [F,h,w,3,64] int32{', zig-zag' if args.zigzag else ''})",
                   "frames_per_gpu": F, "height": H, "width": W, "parallelism": f"frame-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": "fused_encode_kernel<u8,f64,C=1>",
                     "kernel_ms": round(kern_ms, 4), "algorithmic_bytes_per_launch": algo_bytes,
                     "write_ceiling_GBs": round(fill_gbs, 1),
                     "store_pace": {"total_GBs": round(pace_rate, 1),
                                    "late_fraction": round(pace_late, 4),
                                    "note": "clock-paced address-ordered store sweep, rate "
                                            "adapted per launch (DESIGN.md §5)"}},
        "zerorun": {"blocks_per_gpu": nblk, "symbols_per_gpu": nsym,
                    "ms": round(zms, 3), "Mblocks_per_s": round(nblk / zms / 1e3, 1),
                    "note": "ZeroRunCoder.encode of the zig-zag output (count, scan, emit kernels)",
                    "algorithmic_GBs": round((nblk * 256 + nsym * 4) / (zms * 1e-3) / 1e9, 1)},
        "image2symbols": {"ms": round(fms, 3), "Mpixels_per_s": round(px_step / fms / 1e3, 1),
                          "same_length_as_two_step": fused_same,
                          "note": "u8 pixels -> DCT -> quant -> zig-zag -> zero-run symbols fused "
                                  "(count pass + scan + emit pass; 2 x 1 B/px read, 4 B/symbol "
                                  "written)",
                          "algorithmic_GBs": round((px_step + nsym * 4) / (fms * 1e-3) / 1e9, 1)},
        "exchange": {"alphabet": [b0, b1], "bins": b1 - b0 - 1, "symbols": total_syms,
                     "entropy_bits_per_symbol": round(entropy_bits(pmf), 4),
                     "ms": round(exchange_ms, 3),
                     "collective": f"all_reduce + all_gather_into_tensor ({coll_name(dist)})"
                     if dist is not None else "none (1 rank)"},
    }
    del out, frames
    torch.cuda.empty_cache()

    # ---- cfg4: 1080p x 300, +-16 ME + MC + residual DCT + quant ------------------------------
    if not args.no_inter:
        Fi, Hi, Wi, sr = args.inter_frames, 1080, 1920, args.sr
        seq = inter_frames(Fi, Hi, Wi, seed=4 + 1000 * rank, dev=dev)
        mv = torch.empty((Fi - 1, Hi // 8, Wi // 8), dtype=torch.int64, device=dev)
        q = torch.empty((Fi - 1, Hi // 8, Wi // 8, 3, 64), dtype=torch.int32, device=dev)

        def istep():
            D.inter_encode(seq, sr, table, mv, q, zigzag=args.zigzag)

        iwall, ims = timed(dist, istep, args.inter_steps, 1)
        ipx = (Fi - 1) * Hi * Wi
        ivalue = world * ipx * args.inter_steps / iwall / 1e6
        result["inter"] = {
            "metric": "Mpixels/s: 1080p +-16 full-search ME + MC + residual DCT+quant",
            "value": round(ivalue, 1), "unit": "Mpixels/s",
            "ms_per_step": round(iwall / args.inter_steps * 1e3, 3),
            "config": {"workload": f"cfg4: {Fi} frames 1920x1080 u8 luma per GPU, sr={sr}, "
                                   "ME against the previous source frame (open loop)"},
        }
        if rank == 0 and not args.no_cpu:
            host = seq[:2].cpu().numpy()
            mpx, per_cand, _ = cpu_baseline_me(host, sr)
            result["inter"]["cpu_baseline"] = {
                "value": round(mpx, 4), "unit": "Mpixels/s", "cores": 1, "kind": "port",
                "sample": f"reference ME loop (oracle motion_vectors_loop, float64) on 2 block rows "
                          f"of a 1080p pair at sr={sr}; {per_cand * 1e6:.3f} us per valid candidate, "
                          "extrapolated by exact valid-candidate count"}
        del seq, mv, q
        torch.cuda.empty_cache()

    # ---- cfg5: 8K x 120 frames, frame-sharded ME + DCT, one all-gather of histograms ------
    if not args.no_sharded:
        from ivclab_amd.distributed import shard_pairs
        from ivclab_amd import _native as N
        F5, H5, W5, sr5 = args.sharded_frames, 4320, 7680, 16
        a5, b5 = shard_pairs(F5, rank, world)          # this rank's frames incl. the halo
        n5 = max(b5 - a5, 0)
        seq5 = inter_frames(max(n5, 2), H5, W5, seed=5, dev=dev, first=a5)[:n5]
        pairs5 = max(n5 - 1, 0)
        mv5 = torch.empty((max(pairs5, 1), H5 // 8, W5 // 8), dtype=torch.int64, device=dev)
        q5 = torch.empty((max(pairs5, 1), H5 // 8, W5 // 8, 3, 64), dtype=torch.int32, device=dev)
        nmv = (2 * sr5 + 1) ** 2
        hist5 = torch.zeros(HIST_BINS + nmv, dtype=torch.int64, device=dev)

        side = torch.cuda.Stream(device=dev)
        ck = args.sharded_chunk if args.sharded_chunk > 0 else max(pairs5, 1)

        def sstep():
            # the step: ME + MC + residual DCT + quantise of this rank's pairs, then the
            # symbol histograms (coefficients | MV indices) and their all-gather.  The pairs
            # go in chunks of `ck`: ME is VALU-bound and the histogram HBM-bound, so chunk k's
            # histograms run on a side stream while chunk k+1 is encoded (same work, same
            # counts: integer adds in one stream order)
            main = torch.cuda.current_stream()
            L = N.lib()
            prev_wg = L.ivc_histogram_occupancy()
            N.check(L.ivc_set_histogram_occupancy(args.sharded_hist_wg))
            hist5.zero_()
            for p0 in range(0, pairs5, ck):
                p1 = min(p0 + ck, pairs5)
                D.inter_encode(seq5[p0:p1 + 1], sr5, table, mv5[p0:p1], q5[p0:p1],
                               zigzag=args.zigzag, stream=main)
                side.wait_stream(main)
                D.histogram(q5[p0:p1].view(-1), HIST_LO, hist5[:HIST_BINS], stream=side)
                D.histogram(mv5[p0:p1].view(-1), 0, hist5[HIST_BINS:], stream=side)
            main.wait_stream(side)
            N.check(L.ivc_set_histogram_occupancy(prev_wg))
            return global_histogram(hist5)

        swall, _ = timed(dist, sstep, args.sharded_steps, 1)
        g5 = sstep()
        total5 = (F5 - 1) * H5 * W5
        result["sharded"] = {
            "metric": "Mpixels/s: 8K frame-sharded +-16 ME + residual DCT+quant with one "
                      "histogram all-gather (cfg5)",
            "value": round(total5 * args.sharded_steps / swall / 1e6, 1), "unit": "Mpixels/s",
            "scaling": "strong",
            "ms_per_step": round(swall / args.sharded_steps * 1e3, 3),
            "config": {"workload": f"cfg5: {F5} frames {W5}x{H5} u8 luma split across {world} "
                                   f"rank(s) (+1 halo frame each), sr={sr5}",
                       "pairs_per_rank_max": int(max_over_ranks(dist, float(pairs5)))},
            "exchange": {"collective": f"all_gather_into_tensor ({coll_name(dist)})"
                         if dist is not None else "none (1 rank)",
                         "bins": HIST_BINS + nmv,
                         "symbols": int(g5[:HIST_BINS].sum().item()),
                         "motion_vectors": int(g5[HIST_BINS:].sum().item()),
                         "hist_checksum": int((g5 * torch.arange(1, g5.numel() + 1, device=dev))
                                              .sum().item())},
            "chunk_pairs": ck,
        }
        del seq5, mv5, q5
        torch.cuda.empty_cache()

    if rank == 0 and not args.no_cpu:
        host = intra_frames(80, H, W, seed=3, dev=dev).cpu().numpy()
        mpx, n, dt = cpu_baseline_intra(host)
        result["cpu_baseline"] = {
            "value": round(mpx, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": f"oracle (scipy dct + np.round quantise, the reference's algorithm) on {n} "
                      f"whole {W}x{H} frames of the same generator, {dt:.1f} s single-threaded",
            "cpu": cpu_model()}
        if not args.no_cpu_pool:
            pair = inter_frames(2, 1080, 1920, seed=4, dev=dev).cpu().numpy()
            impx, mmpx, P = cpu_baseline_pool(host[:16], pair, args.sr)
            result["cpu_baseline_multicore"] = {
                "intra_value": round(impx, 3), "me_value": round(mmpx, 4), "unit": "Mpixels/s",
                "cores": P, "kind": "port", "cpu": cpu_model(),
                "sample": f"the same oracle paths frame-sharded over {P} worker processes: intra "
                          "on whole 4K frames (~4 s), the ME loop on one 16-row stripe of a "
                          "1080p pair per worker, extrapolated per valid candidate"}

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
