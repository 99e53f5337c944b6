#!/bin/bash
# r05am: symbols -> image, the IDCT's 1/16 folded into the DQ_INT table (d1) vs at the end (d0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/d0.so ab/d1.so ab/d0.so ab/d1.so --rounds 6 --legs symbols2image > gpurun_out/r05am_ab_decode_fold16.log 2>&1 || { tail -20 gpurun_out/r05am_ab_decode_fold16.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05am_ab_decode_fold16.log
