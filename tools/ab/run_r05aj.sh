#!/bin/bash
# r05aj: cost of lds_barrier (the explicit LDS wait before every barrier): pre-fix sources
# (b796e32) vs current, same process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/pre.so ab/cur.so --rounds 6 --legs zerorun_encode,symbols_hist,symbols2image > gpurun_out/r05aj_ab_symbols.log 2>&1 || { tail -20 gpurun_out/r05aj_ab_symbols.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05aj_ab_symbols.log
timeout -k 10 300 python tools/ab/ab_cfg2.py ab/pre.so ab/cur.so --rounds 6 > gpurun_out/r05aj_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r05aj_ab_cfg2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05aj_ab_cfg2.log
timeout -k 10 300 python tools/ab/ab_me.py ab/pre.so ab/cur.so --rounds 6 > gpurun_out/r05aj_ab_me.log 2>&1 || { tail -20 gpurun_out/r05aj_ab_me.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05aj_ab_me.log
