#!/bin/bash
# r05n: single-pass zero-run encoder (decoupled look-back): parity tests, then A/B vs the
# pipelined two-pass form, then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k zerorun --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05n_pytest_zr.log 2>&1 || { tail -40 gpurun_out/r05n_pytest_zr.log; exit 1; }
tail -2 gpurun_out/r05n_pytest_zr.log
timeout -k 10 600 python tools/ab/ab_symbols.py ab/zrbase.so ab/zrcur.so --rounds 4 --legs zerorun_encode > gpurun_out/r05n_ab_zr.log 2>&1 || { tail -20 gpurun_out/r05n_ab_zr.log; exit 1; }
cat gpurun_out/r05n_ab_zr.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05n_pytest.log 2>&1 || { tail -40 gpurun_out/r05n_pytest.log; exit 1; }
tail -2 gpurun_out/r05n_pytest.log
