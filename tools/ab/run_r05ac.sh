#!/bin/bash
# r05ac: image -> symbols pipeline: count / emitter grid fractions (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/ya.so ab/yc6.so ab/yc4.so ab/ye6.so ab/ye4.so --rounds 4 --legs intra_symbols > gpurun_out/r05ac_ab_symbols.log 2>&1 || { tail -20 gpurun_out/r05ac_ab_symbols.log; exit 1; }
cat gpurun_out/r05ac_ab_symbols.log
