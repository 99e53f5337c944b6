#!/bin/bash
# r06w: ME window-energy phase — rows read ahead (EPRE) and an interior-tile path without the frame checks (EFAST)
# (same-process A/B against the base build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_me.py ab/base.so ab/epre4.so ab/efast.so ab/both.so ab/epre8.so --rounds 4 --oracle > gpurun_out/r06w_ab_me_energy.log 2>&1 || { tail -20 gpurun_out/r06w_ab_me_energy.log; exit 1; }
cat gpurun_out/r06w_ab_me_energy.log
