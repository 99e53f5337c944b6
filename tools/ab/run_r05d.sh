#!/bin/bash
# r05d: cfg2 pacing/occupancy A/B; ME sequence comparison (the r05c sharded-histogram verify
# failure); ME PMC of the product (PAIR=0) build; default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab/ab_me_seq.py ab/mebase.so ab/memerge.so ab/mepair.so > gpurun_out/r05d_ab_me_seq.log 2>&1 || { tail -20 gpurun_out/r05d_ab_me_seq.log; exit 1; }
cat gpurun_out/r05d_ab_me_seq.log
timeout -k 10 600 python tools/ab/ab_cfg2.py ab/c3base.so ab/c3pst.so ab/c3w7.so --rounds 3 --pace 0,4500,5800 > gpurun_out/r05d_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r05d_ab_cfg2.log; exit 1; }
cat gpurun_out/r05d_ab_cfg2.log
ME_NO_F64=1 CHILD="tools/me_pmc_child.py" PMC_GROUPS=tools/pmc_groups_me.txt OUTDIR=r05d_pmc_me timeout -k 10 600 bash tools/gpu_pmc_child.sh > gpurun_out/r05d_pmc_me.log 2>&1 || { tail -20 gpurun_out/r05d_pmc_me.log; exit 1; }
echo pmc ok
timeout -k 10 600 python bench.py > gpurun_out/r05d_bench.json 2> gpurun_out/r05d_bench.err || { tail -20 gpurun_out/r05d_bench.err; exit 1; }
python -c "
import json; p=json.load(open('gpurun_out/r05d_bench.json'))
print('headline', p['value'], p['roofline']['frac'])
for k in ['image2symbols','zerorun','decode']: print(k, p[k].get('ms'))
print('inter', p['inter']['ms_per_step'], p['inter']['roofline']['kernel_ms'])
print('cfg2', p['cfg2']['one_frame']['ms_per_launch'], p['cfg2']['batch_64']['ms_per_launch'])
print('sharded', p['sharded']['exchange']['hist_sha256'], p['sharded']['ms_per_step'])
print('verify', p['verify']['ok'], p['verify']['failures_rank0'])
"
