#!/bin/bash
# r06aj: ±16 ME with offset R = 10 split between waves 0 and 1 by M-tile (IVC_ME_BAL: 63, 63,
# 60, 60 matrix steps per wave instead of 66, 60, 60, 60), same-process A/B, vectors compared
# (and with the C oracle on pair 0).  Vectors identical but slower (4.383 -> 4.483 ms: the split
# raises the kernel to the 128-VGPR cap with a spill); the switch was removed after this run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_me.py ab/base.so ab/bal.so --rounds 6 --oracle > gpurun_out/r06aj_ab_me_balance.log 2>&1 || { tail -20 gpurun_out/r06aj_ab_me_balance.log; exit 1; }
cat gpurun_out/r06aj_ab_me_balance.log
