#!/bin/bash
# r05h: pixels -> symbols count-pass occupancy / prefetch A/B (with and without the histogram)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_symbols.py ab/symcur.so ab/symw7.so ab/sympf1.so --rounds 4 --legs intra_symbols,symbols_hist > gpurun_out/r05h_ab_symbols.log 2>&1 || { tail -20 gpurun_out/r05h_ab_symbols.log; exit 1; }
cat gpurun_out/r05h_ab_symbols.log
timeout -k 10 120 ./tools/ubench/tiny_call > gpurun_out/r05h_tiny_call.log 2>&1 || { tail -20 gpurun_out/r05h_tiny_call.log; exit 1; }
tail -3 gpurun_out/r05h_tiny_call.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "tiny or dct or quant" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05h_pytest.log 2>&1 || { tail -30 gpurun_out/r05h_pytest.log; exit 1; }
tail -2 gpurun_out/r05h_pytest.log
