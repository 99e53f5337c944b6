#!/bin/bash
# r06af: where the ±16 ME kernel's time goes after the round-6 energy change (IVC_ME_ABL timing
# builds, vectors wrong on purpose except base: 1 no energies, 4 no staging writes, 5 neither,
# 8 no search), same process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_me.py ab/base.so ab/abl1.so ab/abl4.so ab/abl5.so ab/abl8.so --rounds 4 > gpurun_out/r06af_ab_me_ablation.log 2>&1 || { tail -20 gpurun_out/r06af_ab_me_ablation.log; exit 1; }
cat gpurun_out/r06af_ab_me_ablation.log
