#!/bin/bash
# r06ag: ME window energies with each row's sum of squares formed apart from the prefix (one
# add per row on the chain; IVC_ME_EIND), rows read 4 / 6 / 8 ahead, same-process A/B.
# Slower at 1080p (4.368 -> 4.44 ms); the switch was removed after this run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_me.py ab/base.so ab/eind.so ab/eind6.so ab/eind8.so --rounds 5 --oracle > gpurun_out/r06ag_ab_me_energy_rowsums.log 2>&1 || { tail -20 gpurun_out/r06ag_ab_me_energy_rowsums.log; exit 1; }
cat gpurun_out/r06ag_ab_me_energy_rowsums.log
