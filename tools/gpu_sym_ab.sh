#!/bin/bash
# Symbol-path iteration: the zero-run / fused-symbol parity tests on the working-tree libivc,
# then same-process A/B of ab/*.so variants on the cfg3 symbol legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workload.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "zero or zr or symbol or histogram or image2" > gpurun_out/pytest_sym.log 2>&1 || { tail -30 gpurun_out/pytest_sym.log; exit 1; }
tail -2 gpurun_out/pytest_sym.log
timeout -k 10 500 python -u tools/ab/ab_symbols.py ${AB_LIBS} --rounds 5 > gpurun_out/ab_sym.log 2>&1 || { tail -20 gpurun_out/ab_sym.log; exit 1; }
cat gpurun_out/ab_sym.log
