#!/bin/bash
# r06x: ME window-energy rows from one LDS base per 8 rows (EBASE) on top of EPRE + EFAST
# frame checks (EFAST), same-process A/B against the base build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab/ab_me.py ab/base.so ab/both.so ab/ebase.so ab/ebase6.so --rounds 5 --oracle > gpurun_out/r06x_ab_me_energy_base.log 2>&1 || { tail -20 gpurun_out/r06x_ab_me_energy_base.log; exit 1; }
cat gpurun_out/r06x_ab_me_energy_base.log
