#!/bin/bash
# r05ab: symbols -> image pipeline: EOB-pass workgroups per CU (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/sb.so ab/sc2.so ab/sc4.so ab/sc6.so --rounds 4 --legs symbols2image > gpurun_out/r05ab_ab_decode.log 2>&1 || { tail -20 gpurun_out/r05ab_ab_decode.log; exit 1; }
cat gpurun_out/r05ab_ab_decode.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workload.py -q -x -k "symbols2image or decode" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05ab_pytest.log 2>&1 || { tail -40 gpurun_out/r05ab_pytest.log; exit 1; }
tail -2 gpurun_out/r05ab_pytest.log
