#!/bin/bash
# Zero-run iteration: zero-run parity tests on the working-tree libivc, then same-process A/B
# of ab/*.so variants on the cfg3 zig-zag output.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "zerorun or zero_run or symbols or zw or zr" > gpurun_out/pytest_zr.log 2>&1 || { tail -30 gpurun_out/pytest_zr.log; exit 1; }
tail -2 gpurun_out/pytest_zr.log
timeout -k 10 400 python -u tools/ab/ab_zr.py ${AB_LIBS:-ab/base.so ab/zw2.so} --rounds 5 > gpurun_out/ab_zr.log 2>&1 || { tail -20 gpurun_out/ab_zr.log; exit 1; }
cat gpurun_out/ab_zr.log
