#!/bin/bash
# r06ae: zero-run encode with the int8 hand-off written and read through the caches
# (IVC_ZC_NT=0: the emitter of chunk j reads what the count pass just wrote — can the Infinity
# Cache serve it?) against the non-temporal base, same-process A/B; then the chunk count for
# each build (smaller chunks keep a chunk's hand-off within the 256 MB cache)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r06ae_ab_zerorun_handoff_cached.log
timeout -k 10 300 python tools/ab/ab_zr.py ab/base.so ab/zcnt0.so --rounds 5 > $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 300 python -u tools/ab/chunk_sweep.py --leg zerorun --counts 32,48,64 --rounds 3 --lib ab/base.so >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 300 python -u tools/ab/chunk_sweep.py --leg zerorun --counts 32,48,64 --rounds 3 --lib ab/zcnt0.so >> $O 2>&1 || { tail -20 $O; exit 1; }
cat $O
