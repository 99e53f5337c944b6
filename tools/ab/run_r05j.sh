#!/bin/bash
# r05j: decode float64 work moved to the integer pipe (A/B), tiny calls with kernel-argument
# inputs (ubench + GPU tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_symbols.py ab/decbase.so ab/deccur.so --rounds 4 --legs symbols2image > gpurun_out/r05j_ab_decode.log 2>&1 || { tail -20 gpurun_out/r05j_ab_decode.log; exit 1; }
cat gpurun_out/r05j_ab_decode.log
timeout -k 10 120 ./tools/ubench/tiny_call > gpurun_out/r05j_tiny_call.log 2>&1 || { tail -20 gpurun_out/r05j_tiny_call.log; exit 1; }
tail -3 gpurun_out/r05j_tiny_call.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05j_pytest.log 2>&1 || { tail -40 gpurun_out/r05j_pytest.log; exit 1; }
tail -3 gpurun_out/r05j_pytest.log
