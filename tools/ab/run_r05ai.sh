#!/bin/bash
# r05ai: race probe on one box: merge-next (mn), merge-next + LDS wait before the loop barrier
# (mw), round-4 merge placement (mo); interleaved, 150 reps each pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in mn mw mo mw mn mw; do
  timeout -k 10 300 python -u tools/race_probe.py --reps 150 --quiet --lib ab/$v.so > gpurun_out/r05ai_run.log 2>&1 || { tail -20 gpurun_out/r05ai_run.log; exit 1; }
  grep "runs differ" gpurun_out/r05ai_run.log | tee -a gpurun_out/r05ai_summary.log
done
timeout -k 10 300 python tools/ab/ab_me.py ab/mn.so ab/mw.so ab/mo.so --rounds 5 > gpurun_out/r05ai_ab_me.log 2>&1 || { tail -20 gpurun_out/r05ai_ab_me.log; exit 1; }
cat gpurun_out/r05ai_ab_me.log
