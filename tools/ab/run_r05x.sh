#!/bin/bash
# r05x: zero-run encoder pipeline grid knobs (count / emission workgroups per CU, groups per
# count wave)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_symbols.py ab/zrb.so ab/zrc6.so ab/zrc12.so ab/zre4.so ab/zre8.so ab/zrg2.so --rounds 3 --legs zerorun_encode > gpurun_out/r05x_ab_zr.log 2>&1 || { tail -20 gpurun_out/r05x_ab_zr.log; exit 1; }
cat gpurun_out/r05x_ab_zr.log
