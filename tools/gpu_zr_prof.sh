#!/bin/bash
# Zero-run A/B of ab/*.so variants, then per-kernel rocprofv3 stats of each variant alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab/ab_zr.py ${AB_LIBS} --rounds 4 > gpurun_out/ab_zr.log 2>&1 || { tail -20 gpurun_out/ab_zr.log; exit 1; }
cat gpurun_out/ab_zr.log
for l in ${AB_LIBS}; do
  n=$(basename $l .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/zrprof_$n" -o run -- python tools/ab/ab_zr.py $l --rounds 2 > gpurun_out/zrprof_$n.log 2>&1 || { tail -20 gpurun_out/zrprof_$n.log; exit 1; }
  echo "== $n"
  f=$(find gpurun_out/zrprof_$n -name "*kernel_stats.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
  find gpurun_out/zrprof_$n -name "*kernel_trace.csv" -delete
done
