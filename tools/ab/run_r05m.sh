#!/bin/bash
# r05m: one-wave tiny quantize / zigzag launches (probe, ubench, parity tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/diag_tiny.py > gpurun_out/r05m_diag.log 2>&1 || { cat gpurun_out/r05m_diag.log; exit 1; }
cat gpurun_out/r05m_diag.log
timeout -k 10 120 ./tools/ubench/tiny_call > gpurun_out/r05m_tiny_call.log 2>&1 || { tail -20 gpurun_out/r05m_tiny_call.log; exit 1; }
tail -4 gpurun_out/r05m_tiny_call.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05m_pytest.log 2>&1 || { tail -40 gpurun_out/r05m_pytest.log; exit 1; }
tail -3 gpurun_out/r05m_pytest.log
