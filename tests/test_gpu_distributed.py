"""The multi-rank bench path on one GPU: `bench.py --gpus 2` starts its own two ranks
(torch.distributed.run, 127.0.0.1), both on cuda:0 with the gloo backend (RCCL needs one GPU
per rank; IVC_BENCH_BACKEND=gloo is the rehearsal switch), and runs a small cfg5: each rank
encodes its shard_pairs range, histograms it, and the ranks all-gather.  The gathered
histogram must equal the 1-rank run's, and bench's own verification (sampled pairs against
the C oracle chain, the gathered histogram against one unsharded unchunked run) must pass."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--no-intra", "--no-symbols", "--no-inter", "--no-class-api", "--no-cpu",
         "--steps", "1", "--warmup", "1", "--sharded-frames", "9", "--sharded-height", "272",
         "--sharded-width", "480", "--sharded-steps", "2", "--sharded-chunk", "2"]


def run_bench(n):
    env = dict(os.environ, IVC_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)] + SMALL,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_gloo_equals_one_rank():
    one = run_bench(1)
    two = run_bench(2)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    for res in (one, two):
        assert res["verify"]["ok"], res["verify"]
    s1, s2 = one["sharded"], two["sharded"]
    assert s2["exchange"]["collective"].startswith("all_gather_into_tensor (gloo")
    assert s2["config"]["pairs_per_rank_max"] == 4 and s1["config"]["pairs_per_rank_max"] == 8
    for k in ("hist_sha256", "hist_checksum", "symbols", "motion_vectors"):
        assert s2["exchange"][k] == s1["exchange"][k], k
    assert s1["exchange"]["motion_vectors"] == 8 * (272 // 8) * (480 // 8)


RCCL_CHILD = r"""
import json, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, {root!r})
from ivclab_amd.distributed import init_single_rank, global_bounds, global_histogram
import ivclab_amd.device as D
from oracle import ivc_oracle as O
torch.cuda.set_device(0)
init_single_rank("cuda:0")
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
rng = np.random.default_rng(11)
host = rng.integers(-300, 301, 1 << 20).astype(np.int32)
host[::97] = 4000
sym = torch.from_numpy(host).cuda()
lo = -400
hist = torch.zeros(4402, dtype=torch.int64, device="cuda")
D.histogram(sym, lo, hist)
g = global_histogram(hist, force=True)            # one RCCL all-gather on the device tensor
mm = torch.empty(2, dtype=torch.int32, device="cuda")
D.minmax(sym, mm)
b = global_bounds(mm, force=True)                 # one RCCL all-reduce
torch.cuda.synchronize()
want = O.histogram(host, lo, 4402)
out = dict(rccl_equals_local=bool(torch.equal(g, hist)),
           equals_oracle=bool(np.array_equal(g.cpu().numpy(), want)),
           bounds=list(b), want_bounds=[int(host.min()), int(host.max())],
           g_is_new=g.data_ptr() != hist.data_ptr())
dist.destroy_process_group()
print(json.dumps(out))
"""


def test_rccl_single_rank_exchange():
    """The exchange's collectives through RCCL itself on a one-GPU box: a fresh process
    creates a one-rank "nccl" (= RCCL) group on cuda:0 before any other GPU call, and
    global_histogram / global_bounds are forced past their one-rank shortcut
    (ivclab_amd/distributed.py), so `all_gather_into_tensor` and `all_reduce` run on device
    tensors.  The gathered histogram equals the local one and the oracle's."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", RCCL_CHILD.format(root=ROOT)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["rccl_equals_local"] and out["equals_oracle"] and out["g_is_new"], out
    assert out["bounds"] == out["want_bounds"], out


def test_bench_rccl_world1_equals_one_rank():
    """`bench.py --rccl` at one rank runs the cfg5 histogram exchange through a one-rank RCCL
    group: the collective is reported as RCCL and the histogram equals the plain run's."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    res = []
    for extra in ([], ["--rccl"]):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] +
                           SMALL + extra, cwd=ROOT, env=env, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        res.append(json.loads(lines[-1]))
    plain, rccl = res
    assert rccl["verify"]["ok"], rccl["verify"]
    assert plain["sharded"]["exchange"]["collective"] == "none (1 rank)"
    assert rccl["sharded"]["exchange"]["collective"] == "all_gather_into_tensor (RCCL, 1 rank)"
    for k in ("hist_sha256", "hist_checksum", "symbols", "motion_vectors"):
        assert rccl["sharded"]["exchange"][k] == plain["sharded"]["exchange"][k], k
