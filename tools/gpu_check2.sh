#!/bin/bash
# Full GPU parity suite, smoke, then the default bench line (with its in-run PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG:-chk}.json 2> gpurun_out/bench_${TAG:-chk}.err || { tail -20 gpurun_out/bench_${TAG:-chk}.err; exit 1; }
python -c "
import json,sys
d=json.loads(open('gpurun_out/bench_${TAG:-chk}.json').read().strip().splitlines()[-1])
print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'],'traffic',d['roofline'].get('traffic'),d['roofline'].get('traffic_detail'))
for k in ('inter','inter_f64','sharded','zerorun','image2symbols'):
    if k in d: print(k, d[k].get('value', d[k].get('ms')), d[k].get('ms_per_step'), d[k].get('roofline',{}).get('frac'))
print('verify', d.get('verify',{}).get('ok'), d.get('verify',{}).get('failures_rank0'), 'wall', d.get('bench_wall_s'))
"
