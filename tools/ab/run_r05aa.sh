#!/bin/bash
# r05aa: zero-run emission at 5 workgroups per CU, confirmation A/B
# count wave)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_symbols.py ab/zb.so ab/ze5.so ab/ze5c7.so ab/ze5c6.so --rounds 5 --legs zerorun_encode > gpurun_out/r05aa_ab_zr.log 2>&1 || { tail -20 gpurun_out/r05aa_ab_zr.log; exit 1; }
cat gpurun_out/r05aa_ab_zr.log
