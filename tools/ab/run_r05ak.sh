#!/bin/bash
# r05ak: zero-run pipeline: int8 hand-off through the Infinity Cache? (nt vs temporal stores and
# loads of the hand-off, 32 / 48 / 64 chunks)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/zb.so ab/zk64.so ab/zt.so ab/zt64.so ab/zt48.so --rounds 6 --legs zerorun_encode > gpurun_out/r05ak_ab_zerorun.log 2>&1 || { tail -20 gpurun_out/r05ak_ab_zerorun.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05ak_ab_zerorun.log
