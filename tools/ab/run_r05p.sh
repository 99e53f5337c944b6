#!/bin/bash
# r05p: zero-run emission slots with 4 mbcnt + a shift-add (A/B), tiny-call Python paths
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/zslot0.so ab/zslot1.so --rounds 5 --legs zerorun_encode > gpurun_out/r05p_ab_zr.log 2>&1 || { tail -20 gpurun_out/r05p_ab_zr.log; exit 1; }
cat gpurun_out/r05p_ab_zr.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "zerorun or tiny or quant" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05p_pytest.log 2>&1 || { tail -30 gpurun_out/r05p_pytest.log; exit 1; }
tail -2 gpurun_out/r05p_pytest.log
timeout -k 10 300 python tools/small_call_probe.py > gpurun_out/r05p_small.log 2>&1 || { tail -20 gpurun_out/r05p_small.log; exit 1; }
cat gpurun_out/r05p_small.log
