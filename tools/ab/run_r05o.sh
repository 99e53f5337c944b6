#!/bin/bash
# r05o: single-pass zero-run encoder tile size / occupancy A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_symbols.py ab/zrbase.so ab/zrg4.so ab/zrg2.so ab/zrg1.so --rounds 4 --legs zerorun_encode > gpurun_out/r05o_ab_zr.log 2>&1 || { tail -20 gpurun_out/r05o_ab_zr.log; exit 1; }
cat gpurun_out/r05o_ab_zr.log
