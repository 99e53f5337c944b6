#!/bin/bash
# r05v: ME segments down a column strip with the shared reference rows carried in LDS (A/B
# over the segment length), ME parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workload.py -q -x -k "me_ or motion or inter" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05v_pytest_me.log 2>&1 || { tail -40 gpurun_out/r05v_pytest_me.log; exit 1; }
tail -2 gpurun_out/r05v_pytest_me.log
timeout -k 10 900 python tools/ab/ab_me.py ab/meold.so ab/mek9.so ab/mek17.so ab/mek5.so --rounds 4 --oracle > gpurun_out/r05v_ab_me.log 2>&1 || { tail -20 gpurun_out/r05v_ab_me.log; exit 1; }
cat gpurun_out/r05v_ab_me.log
