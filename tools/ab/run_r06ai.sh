#!/bin/bash
# r06ai: pixels -> symbols (+ histogram) chunk count re-swept on the round-6 sources
# (tuning API, one process, outputs compared)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r06ai_sweep_symbols_chunks.log
timeout -k 10 600 python -u tools/ab/chunk_sweep.py --leg symbols_hist --counts 8,12,16,20,24 --rounds 4 > $O 2>&1 || { tail -20 $O; exit 1; }
cat $O
