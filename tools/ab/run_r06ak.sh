#!/bin/bash
# r06ak: symbols -> image with clock-paced image stores (IVC_DEC_PACE_WGBPS: the write rate of
# the schedule, 3.6-4.2 TB/s of writes = ~5.7-6.7 TB/s of total traffic at the call's mix)
# against the unpaced base, same-process A/B, images compared.  Every rate slower (17.95 ->
# 18.6-28.9 ms): the decode cannot keep a store schedule; removed after this run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/base.so ab/p36.so ab/p38.so ab/p40.so ab/p42.so --rounds 4 --legs symbols2image > gpurun_out/r06ak_ab_decode_paced.log 2>&1 || { tail -20 gpurun_out/r06ak_ab_decode_paced.log; exit 1; }
cat gpurun_out/r06ak_ab_decode_paced.log
