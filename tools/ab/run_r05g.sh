#!/bin/bash
# r05g: cfg2 and ME A/B of the current build against round 4, GPU tests, smoke, bench,
# tiny-call ubench (completion signalled by the op kernel itself)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab/ab_cfg2.py ab/c3base.so ab/cur.so --rounds 4 --pace 0 > gpurun_out/r05g_ab_cfg2.log 2>&1 || { tail -20 gpurun_out/r05g_ab_cfg2.log; exit 1; }
cat gpurun_out/r05g_ab_cfg2.log
timeout -k 10 600 python tools/ab/ab_me.py ab/mebase.so ab/cur.so ab/mett.so --rounds 4 --oracle > gpurun_out/r05g_ab_me.log 2>&1 || { tail -20 gpurun_out/r05g_ab_me.log; exit 1; }
cat gpurun_out/r05g_ab_me.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05g_pytest.log 2>&1 || { tail -40 gpurun_out/r05g_pytest.log; exit 1; }
tail -3 gpurun_out/r05g_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05g_smoke.log 2>&1 || { tail -20 gpurun_out/r05g_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > gpurun_out/r05g_bench.json 2> gpurun_out/r05g_bench.err || { tail -20 gpurun_out/r05g_bench.err; exit 1; }
python -c "
import json; p=json.load(open('gpurun_out/r05g_bench.json'))
print('headline', p['value'], p['roofline']['frac'])
for k in ['image2symbols','zerorun','decode']: print(k, p[k].get('ms'))
print('inter', p['inter']['ms_per_step'], p['inter']['roofline']['kernel_ms'])
print('cfg2', p['cfg2']['one_frame']['ms_per_launch'], p['cfg2']['batch_64']['ms_per_launch'])
print('small', p['class_api']['small_call'])
print('sharded', p['sharded']['exchange']['hist_sha256'], p['sharded']['ms_per_step'])
print('verify', p['verify']['ok'], p['verify']['failures_rank0'])
"
timeout -k 10 120 ./tools/ubench/tiny_call > gpurun_out/r05g_tiny_call.log 2>&1 || { tail -20 gpurun_out/r05g_tiny_call.log; exit 1; }
tail -3 gpurun_out/r05g_tiny_call.log
