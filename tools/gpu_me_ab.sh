#!/bin/bash
# ME iteration: ME/inter parity tests on the working-tree libivc, then same-process A/B of
# ab/*.so variants on the cfg4 (1080p x 300) and cfg5-shaped (8K x 24) inter chains.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workload.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "me_ or motion or inter or mv or sequence or cfg4 or cfg5 or chain" > gpurun_out/pytest_me.log 2>&1 || { tail -30 gpurun_out/pytest_me.log; exit 1; }
tail -2 gpurun_out/pytest_me.log
timeout -k 10 400 python -u tools/ab/ab_intra.py ${AB_LIBS:-ab/base.so ab/tileB.so ab/tileA.so} --frames 4 --rounds 5 --inter > gpurun_out/ab_me.log 2>&1 || { tail -20 gpurun_out/ab_me.log; exit 1; }
grep inter gpurun_out/ab_me.log
timeout -k 10 400 python -u tools/ab/ab_intra.py ${AB_LIBS:-ab/base.so ab/tileB.so ab/tileA.so} --frames 4 --rounds 3 --inter --inter-shape 24x4320x7680 > gpurun_out/ab_me8k.log 2>&1 || { tail -20 gpurun_out/ab_me8k.log; exit 1; }
grep inter gpurun_out/ab_me8k.log
