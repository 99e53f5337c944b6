#!/bin/bash
# r05w: symbols -> image parse stores without exec-mask branches (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/dnb0.so ab/dnb1.so --rounds 5 --legs symbols2image > gpurun_out/r05w_ab_decode.log 2>&1 || { tail -20 gpurun_out/r05w_ab_decode.log; exit 1; }
cat gpurun_out/r05w_ab_decode.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workload.py -q -x -k "symbols2image or decode" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05w_pytest.log 2>&1 || { tail -40 gpurun_out/r05w_pytest.log; exit 1; }
tail -2 gpurun_out/r05w_pytest.log
