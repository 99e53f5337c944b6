#!/bin/bash
# r05ap: cfg2 C = 3 encoder: quantiser table out of LDS (read from the kernel argument in the
# rare exact-division fallback: 19,968 B of LDS) with 8 waves per SIMD (5 VGPRs spill) vs current
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab/ab_cfg2.py ab/cb.so ab/ck8.so ab/cb.so ab/ck8.so --rounds 6 > gpurun_out/r05ap_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r05ap_ab_cfg2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05ap_ab_cfg2.log
