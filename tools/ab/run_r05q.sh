#!/bin/bash
# r05q: tiny quantise with a device table copy; small-call breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "tiny or quant or dct" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05q_pytest.log 2>&1 || { tail -30 gpurun_out/r05q_pytest.log; exit 1; }
tail -2 gpurun_out/r05q_pytest.log
timeout -k 10 120 ./tools/ubench/tiny_call > gpurun_out/r05q_tiny_call.log 2>&1 || { tail -20 gpurun_out/r05q_tiny_call.log; exit 1; }
tail -3 gpurun_out/r05q_tiny_call.log
timeout -k 10 300 python tools/small_call_breakdown.py > gpurun_out/r05q_breakdown.log 2>&1 || { tail -20 gpurun_out/r05q_breakdown.log; exit 1; }
cat gpurun_out/r05q_breakdown.log
timeout -k 10 300 python tools/small_call_probe.py > gpurun_out/r05q_small.log 2>&1 || { tail -20 gpurun_out/r05q_small.log; exit 1; }
cat gpurun_out/r05q_small.log
