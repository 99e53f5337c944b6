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
