#!/bin/bash
# r05ar: symbols -> image default chunking: 32 chunks / 16 K-tile minimum (s32) vs 64 / 13 K (s64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/s32.so ab/s64.so --rounds 8 --legs symbols2image > gpurun_out/r05ar_ab.log 2>&1 || { tail -20 gpurun_out/r05ar_ab.log; exit 1; }
timeout -k 10 600 python tools/ab/ab_symbols.py ab/s32.so ab/s64.so --rounds 8 --frames 64 --legs symbols2image >> gpurun_out/r05ar_ab.log 2>&1 || { tail -20 gpurun_out/r05ar_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05ar_ab.log
