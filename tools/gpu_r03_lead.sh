#!/bin/bash
# Store-pace schedule-origin lead A/B (IVC_PACE_LEAD ticks of 10 ns) on the headline leg alone,
# one bench process per lead on the same box; then the round's rocprofv3 kernel-trace summary
# of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
INTRA_ONLY="--no-inter --no-symbols --no-class-api --no-sharded --no-cpu --no-pmc --no-luma --no-verify"
for lead in ${LEADS:-300 1500 5000 300}; do
  IVC_PACE_LEAD=$lead timeout -k 10 300 python bench.py --steps 20 --warmup 5 $INTRA_ONLY > gpurun_out/lead_$lead.json 2> gpurun_out/lead_$lead.err || { tail -5 gpurun_out/lead_$lead.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('gpurun_out/lead_$lead.json')); r=d['roofline']; p=r['store_pace']
t=p['trace_timed']; import statistics as S
print('lead $lead frac', r['frac'], 'ms', r['kernel_ms'], 'settled', p['settled_GBs'], 'over', p['launches_over_late_threshold'],
      'late_startup_mean', round(S.mean(x[6] for x in t),4), 'late_mean', round(S.mean(x[1] for x in t),4), 'lag', round(S.mean(x[3] for x in t),1))"
done
if [ -n "$PROF" ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r03" -o run -- python bench.py --no-cpu --no-pmc > gpurun_out/prof_r03.log 2>&1 || { tail -20 gpurun_out/prof_r03.log; exit 1; }
  python tools/prof_summary.py gpurun_out/prof_r03 gpurun_out/r03_bench_kernels.md "rocprofv3 --kernel-trace --stats -- python bench.py --no-cpu --no-pmc" || true
  find gpurun_out/prof_r03 -name "*kernel_trace.csv" -delete
  head -30 gpurun_out/r03_bench_kernels.md
fi
