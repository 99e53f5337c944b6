#!/bin/bash
# r06ab: symbols -> image with the EOB pass's stream loads cached (IVC_ZF_TEMPORAL=1, ab/zft.so)
# so the parse's second read can hit the Infinity Cache, unthrottled and with the EOB pass held
# L chunks ahead of the decode (IVC_TUNE_S2I_LAG = L + 1), against the non-temporal base build.
# No setting was faster (profiles/r06ab_sweep_decode_zf_cached.log); the variant macro and the
# throttle were removed after this run (chunk_sweep.py --lags needs them).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r06ab_sweep_decode_zf_cached.log
timeout -k 10 300 python -u tools/ab/chunk_sweep.py --leg symbols2image --counts 64,128 --lags 1,5,9 --rounds 3 --lib ab/base.so > $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 300 python -u tools/ab/chunk_sweep.py --leg symbols2image --counts 64,128 --lags 1,3,5,9 --rounds 3 --lib ab/zft.so >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 300 python -u tools/ab/chunk_sweep.py --leg symbols2image --counts 64,128 --lags 1,5,9 --rounds 3 --lib ab/base.so >> $O 2>&1 || { tail -20 $O; exit 1; }
cat $O
