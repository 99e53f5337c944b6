#!/bin/bash
# r06ao: the evidence run's failing PMC pass repeated (bench under rocprofv3 --pmc WRITE_SIZE,
# whose verify reported cfg2 frames 0 / 63 once), six times, with the verify naming how many elements
# differ and where; then once more plain
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4 5 6; do
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r06ao_pmc$i" -o run -- python bench.py --steps 3 --warmup 1 --no-inter --no-cpu --no-pmc > gpurun_out/r06ao_pmc$i.log 2>&1; echo "pmc pass $i rc=$?"
  python -c "
import json
t=open('gpurun_out/r06ao_pmc$i.log').read(); i=t.find('{\"metric\"'); r=json.loads(t[i:t.find(chr(10),i)])
print(json.dumps(r['verify']['failures_rank0']), r['cfg2']['batch_64']['ms_per_launch'])
" || true
done
