#!/bin/bash
# r05k: tiny calls with kernel-argument inputs (probe, ubench, GPU tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/diag_tiny.py > gpurun_out/r05k_diag.log 2>&1 || { cat gpurun_out/r05k_diag.log; exit 1; }
cat gpurun_out/r05k_diag.log
timeout -k 10 120 ./tools/ubench/tiny_call > gpurun_out/r05k_tiny_call.log 2>&1 || { tail -20 gpurun_out/r05k_tiny_call.log; exit 1; }
tail -3 gpurun_out/r05k_tiny_call.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05k_pytest.log 2>&1 || { tail -40 gpurun_out/r05k_pytest.log; exit 1; }
tail -3 gpurun_out/r05k_pytest.log
