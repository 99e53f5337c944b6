#!/bin/bash
# r05s: C = 3 encoder's last partial round as (group, plane) items (A/B), 3-channel parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_cfg2.py ab/c3t0.so ab/c3t1.so --rounds 5 --pace 0 > gpurun_out/r05s_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r05s_ab_cfg2.log; exit 1; }
cat gpurun_out/r05s_ab_cfg2.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05s_pytest.log 2>&1 || { tail -40 gpurun_out/r05s_pytest.log; exit 1; }
tail -2 gpurun_out/r05s_pytest.log
