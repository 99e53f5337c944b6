#!/bin/bash
# r05ad: image -> symbols pipeline: count / emitter count-grid fraction, finer (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/ya.so ab/yc7.so ab/yc6.so ab/yc5.so ab/yc3.so --rounds 8 --legs intra_symbols > gpurun_out/r05ad_ab_symbols.log 2>&1 || { tail -20 gpurun_out/r05ad_ab_symbols.log; exit 1; }
cat gpurun_out/r05ad_ab_symbols.log
