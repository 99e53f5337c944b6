#!/bin/bash
# r05a: GPU tests + smoke + default bench on the round-5 cleanup (tuning API, dead ME variants
# removed, pipelined-emitter histogram gated)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_pytest.log 2>&1 || { tail -40 gpurun_out/r05a_pytest.log; exit 1; }
tail -3 gpurun_out/r05a_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a_smoke.log 2>&1 || { tail -20 gpurun_out/r05a_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err || { tail -20 gpurun_out/r05a_bench.err; exit 1; }
python -c "
import json; p=json.load(open('gpurun_out/r05a_bench.json'))
print('headline', p['value'], p['roofline']['frac'])
for k in ['image2symbols','zerorun','decode']: print(k, p[k].get('ms'))
print('inter', p['inter']['ms_per_step'], p['inter']['roofline']['kernel_ms'])
print('cfg2', p['cfg2']['one_frame']['ms_per_launch'], p['cfg2']['batch_64']['ms_per_launch'])
print('small', p['class_api']['small_call'])
"
