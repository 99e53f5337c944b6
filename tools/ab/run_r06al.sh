#!/bin/bash
# r06al: zero-run encode with the pipelined emission's stores on a clock schedule
# (IVC_ZC_PACE_GBPS: 5.6 / 5.9 / 6.2 TB/s of the call's total traffic) against the unpaced
# base, same-process A/B, symbols and offsets compared.  Slower at every rate (10.23 -> 11.35 /
# 11.36 / 16.42 ms); removed after this run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_zr.py ab/base.so ab/z56.so ab/z59.so ab/z62.so --rounds 5 > gpurun_out/r06al_ab_zerorun_paced.log 2>&1 || { tail -20 gpurun_out/r06al_ab_zerorun_paced.log; exit 1; }
cat gpurun_out/r06al_ab_zerorun_paced.log
