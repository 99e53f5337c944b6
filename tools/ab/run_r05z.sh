#!/bin/bash
# r05z: zero-run pipeline: count occupancy, chunk count, emission occupancy (A/B)
# count wave)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_symbols.py ab/zb.so ab/zc4.so ab/zc6.so ab/zk24.so ab/zk40.so ab/ze5.so --rounds 3 --legs zerorun_encode > gpurun_out/r05z_ab_zr.log 2>&1 || { tail -20 gpurun_out/r05z_ab_zr.log; exit 1; }
cat gpurun_out/r05z_ab_zr.log
