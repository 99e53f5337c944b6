"""Multi-process (gloo, CPU) checks of the frame sharding and the histogram exchange used
by the multi-GPU path.  The per-rank histograms here come from the oracle on each rank's
own synthetic symbols; on GPUs they come from libivc's histogram kernel (same bins)."""
import os
import socket

import numpy as np
import pytest

from ivclab_amd.distributed import global_histogram, shard_pairs, shard_range


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 120, 300, 301):
        for world in (1, 2, 3, 8):
            got = [shard_range(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            for (a, b), (c, d) in zip(got, got[1:]):
                assert b == c
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1


def test_shard_pairs_halo():
    for F in (2, 3, 120, 300):
        for world in (1, 2, 4, 8):
            pairs = []
            for r in range(world):
                a, b = shard_pairs(F, r, world)
                pairs += [(f - 1, f) for f in range(a + 1, b)]
            assert pairs == [(f - 1, f) for f in range(1, F)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from oracle import ivc_oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(100 + rank)
        sym = rng.integers(-50, 50, 4096 + 17 * rank).astype(np.int32)
        local = torch.from_numpy(O.histogram(sym, -64, 128))
        total = global_histogram(local)
        q.put((rank, total.numpy().tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_histogram_gloo(world):
    import torch.multiprocessing as mp
    from oracle import ivc_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = sum(O.histogram(np.random.default_rng(100 + r).integers(-50, 50, 4096 + 17 * r)
                           .astype(np.int32), -64, 128) for r in range(world))
    for r in range(world):
        assert results[r] == want.tolist()


def _seq(F, H, W, seed=7):
    """A small synthetic sequence: a smooth texture shifted by a per-frame motion, +-2 noise
    (the shape of bench.inter_frames, on the CPU)."""
    rng = np.random.default_rng(seed)
    lo = rng.integers(0, 256, (H // 4 + 8, W // 4 + 8)).astype(np.float64)
    base = np.kron(lo, np.ones((4, 4)))
    out = []
    for f in range(F):
        dy, dx = (f % 5) - 2, (2 * f % 7) - 3
        fr = base[8 + dy:8 + dy + H, 8 + dx:8 + dx + W] + np.random.default_rng(seed * 31 + f).integers(-2, 3, (H, W))
        out.append(np.clip(fr, 0, 255).astype(np.uint8))
    return np.stack(out)


def _sharded_worker(rank, world, port, q, F, H, W, sr):
    """One rank of the cfg5 pipeline on the CPU: its shard_pairs range (with the halo frame),
    the oracle's inter chain per pair, the coefficient | MV histograms, one all-gather."""
    import torch
    import torch.distributed as dist
    from oracle import ivc_oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seq = _seq(F, H, W)
        a, b = shard_pairs(F, rank, world)
        nmv = (2 * sr + 1) ** 2
        hist = np.zeros(8192 + nmv, np.int64)
        for f in range(a + 1, b):
            mv, qc = O.inter_encode(seq[f - 1], seq[f], sr, 1.0)
            hist[:8192] += O.histogram(qc, -4096, 8192)
            hist[8192:] += O.histogram(mv, 0, nmv)
        total = global_histogram(torch.from_numpy(hist))
        q.put((rank, total.numpy().tolist(), b - a))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_pipeline_equals_unsharded_gloo(world):
    """shard_pairs + per-rank inter coding + global_histogram (the cfg5 step's data flow)
    gives every rank exactly the histogram of the unsharded sequence."""
    import torch.multiprocessing as mp
    from oracle import ivc_oracle as O
    F, H, W, sr = 7, 32, 48, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, F, H, W, sr))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, h, nframes = q.get(timeout=180)
        results[r] = (h, nframes)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seq = _seq(F, H, W)
    nmv = (2 * sr + 1) ** 2
    want = np.zeros(8192 + nmv, np.int64)
    for f in range(1, F):
        mv, qc = O.inter_encode(seq[f - 1], seq[f], sr, 1.0)
        want[:8192] += O.histogram(qc, -4096, 8192)
        want[8192:] += O.histogram(mv, 0, nmv)
    assert sum(n - 1 for _, n in results.values()) == F - 1      # every pair exactly once
    for r in range(world):
        assert results[r][0] == want.tolist()


def test_bench_launcher_and_rank_checks(monkeypatch):
    """bench.py --gpus N without WORLD_SIZE starts N ranks through torch.distributed.run on
    127.0.0.1 with the same arguments; under a launcher, WORLD_SIZE must equal --gpus."""
    import bench
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "3"], 29511)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "--master-port=29511" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit):
        bench.dist_setup(4)
    with pytest.raises(SystemExit):
        bench.parse(["--sharded-hist-wg", "17"])
    n, aff, quota = bench.cpu_share()
    assert 1 <= n <= aff and (quota is None or n <= max(1, quota))
