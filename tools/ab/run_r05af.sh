#!/bin/bash
# r05af: race probe, more reps per mode, with the SSDs of mismatching candidates
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in chunked noside unchunked; do
  timeout -k 10 300 python -u tools/race_probe.py --reps 40 --mode $m > gpurun_out/r05af_$m.log 2>&1 || { tail -20 gpurun_out/r05af_$m.log; exit 1; }
  grep -v "^rep .*hist ok$" gpurun_out/r05af_$m.log | tail -30
done
