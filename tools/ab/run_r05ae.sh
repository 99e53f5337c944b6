#!/bin/bash
# r05ae: cfg5 step repeated, bitwise against an unchunked single-stream run (race probe)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/race_probe.py --reps 12 --mode chunked > gpurun_out/r05ae_plain.log 2>&1 || { tail -20 gpurun_out/r05ae_plain.log; exit 1; }
tail -3 gpurun_out/r05ae_plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05ae_prof" -o run -- python -u tools/race_probe.py --reps 12 --mode chunked > gpurun_out/r05ae_prof_chunked.log 2>&1 || { tail -20 gpurun_out/r05ae_prof_chunked.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r05ae_prof_chunked.log | tail -40
rm -rf gpurun_out/r05ae_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r05ae_prof" -o run -- python -u tools/race_probe.py --reps 8 --mode unchunked > gpurun_out/r05ae_prof_unchunked.log 2>&1 || { tail -20 gpurun_out/r05ae_prof_unchunked.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/r05ae_prof_unchunked.log | tail -30
rm -rf gpurun_out/r05ae_prof
