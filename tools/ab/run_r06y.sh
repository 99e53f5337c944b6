#!/bin/bash
# r06y: symbols -> image with the EOB pass throttled to L chunks ahead of the decode
# (IVC_TUNE_S2I_LAG = L + 1; 1 = unthrottled), crossed with the chunk count; outputs compared.
# Measured slower at every lag (profiles/r06y_sweep_decode_lag.log); the throttle and its
# tuning key were removed again after this run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab/chunk_sweep.py --leg symbols2image --counts 64,128,256 --lags 1,2,3,4 --rounds 3 > gpurun_out/r06y_sweep_decode_lag.log 2>&1 || { tail -20 gpurun_out/r06y_sweep_decode_lag.log; exit 1; }
cat gpurun_out/r06y_sweep_decode_lag.log
