#!/bin/bash
# r05b: GPU tests + smoke + default bench, then the cfg2 C=3 plane-store A/B and PMC of both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_cfg2.py ab/c3base.so ab/c3pst.so --rounds 5 > gpurun_out/r05b_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r05b_ab_cfg2.log; exit 1; }
cat gpurun_out/r05b_ab_cfg2.log
for v in c3base c3pst; do
  CHILD="tools/cfg2_pmc_child.py ab/$v.so" PMC_GROUPS=tools/pmc_groups_luma.txt OUTDIR=r05b_pmc_$v timeout -k 10 600 bash tools/gpu_pmc_child.sh > gpurun_out/r05b_pmc_$v.log 2>&1 || { tail -20 gpurun_out/r05b_pmc_$v.log; exit 1; }
done
echo pmc ok
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05b_pytest.log 2>&1 || { tail -40 gpurun_out/r05b_pytest.log; exit 1; }
tail -3 gpurun_out/r05b_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b_smoke.log 2>&1 || { tail -20 gpurun_out/r05b_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err || { tail -20 gpurun_out/r05b_bench.err; exit 1; }
python -c "
import json; p=json.load(open('gpurun_out/r05b_bench.json'))
print('headline', p['value'], p['roofline']['frac'])
for k in ['image2symbols','zerorun','decode']: print(k, p[k].get('ms'))
print('inter', p['inter']['ms_per_step'], p['inter']['roofline']['kernel_ms'])
print('cfg2', p['cfg2']['one_frame']['ms_per_launch'], p['cfg2']['batch_64']['ms_per_launch'])
print('small', p['class_api']['small_call'])
"
