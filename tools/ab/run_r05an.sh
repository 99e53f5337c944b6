#!/bin/bash
# r05an: symbols -> image parse: neighbour symbols by DPP wave shifts (n1) vs strided LDS reads (n0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_symbols.py ab/n0.so ab/n1.so ab/n0.so ab/n1.so --rounds 6 --legs symbols2image > gpurun_out/r05an_ab_decode_nbr_dpp.log 2>&1 || { tail -20 gpurun_out/r05an_ab_decode_nbr_dpp.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05an_ab_decode_nbr_dpp.log
