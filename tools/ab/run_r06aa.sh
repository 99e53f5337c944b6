#!/bin/bash
# r06aa: cfg2 store cache policy (IVC_STORE_AUX 0 / 2 (base: nt) / 3) and the C = 3 kernel's
# minimum waves per SIMD (IVC_C3_WAVES 6 / 8), same-process A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_cfg2.py ab/base.so ab/aux0.so ab/aux3.so ab/c3w6.so ab/c3w8.so --rounds 5 > gpurun_out/r06aa_ab_cfg2_aux_waves.log 2>&1 || { tail -20 gpurun_out/r06aa_ab_cfg2_aux_waves.log; exit 1; }
cat gpurun_out/r06aa_ab_cfg2_aux_waves.log
