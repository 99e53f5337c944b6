#!/bin/bash
# r05aq: chunk-count sweeps of the pipelined calls on the round-5 kernels (tuning API, one process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab/chunk_sweep.py --leg symbols2image --counts 16,24,32,48,64 --rounds 5 > gpurun_out/r05aq_sweep.log 2>&1 || { tail -20 gpurun_out/r05aq_sweep.log; exit 1; }
timeout -k 10 400 python tools/ab/chunk_sweep.py --leg zerorun --counts 16,24,32,48,63 --rounds 5 >> gpurun_out/r05aq_sweep.log 2>&1 || { tail -20 gpurun_out/r05aq_sweep.log; exit 1; }
timeout -k 10 400 python tools/ab/chunk_sweep.py --leg symbols_hist --counts 8,12,16,24,32 --rounds 5 >> gpurun_out/r05aq_sweep.log 2>&1 || { tail -20 gpurun_out/r05aq_sweep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05aq_sweep.log
