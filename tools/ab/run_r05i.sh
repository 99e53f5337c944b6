#!/bin/bash
# r05i: tiny-call ubench (kernel-argument inputs), symbol count-pass occupancy A/B on the new
# one-tile-ahead default, bench (cfg2 batch warm-up)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/tiny_call > gpurun_out/r05i_tiny_call.log 2>&1 || { tail -20 gpurun_out/r05i_tiny_call.log; exit 1; }
cat gpurun_out/r05i_tiny_call.log
timeout -k 10 900 python tools/ab/ab_symbols.py ab/symcur.so ab/symw7.so ab/symw6.so --rounds 4 --legs intra_symbols,symbols_hist,zerorun_encode > gpurun_out/r05i_ab_symbols.log 2>&1 || { tail -20 gpurun_out/r05i_ab_symbols.log; exit 1; }
cat gpurun_out/r05i_ab_symbols.log
timeout -k 10 600 python bench.py > gpurun_out/r05i_bench.json 2> gpurun_out/r05i_bench.err || { tail -20 gpurun_out/r05i_bench.err; exit 1; }
python -c "
import json; p=json.load(open('gpurun_out/r05i_bench.json'))
print('headline', p['value'], p['roofline']['frac'])
for k in ['image2symbols','zerorun','decode']: print(k, p[k].get('ms'))
print('inter', p['inter']['ms_per_step'], p['inter']['roofline']['kernel_ms'])
print('cfg2', p['cfg2']['one_frame']['ms_per_launch'], p['cfg2']['batch_64']['ms_per_launch'])
print('small', p['class_api']['small_call'])
print('verify', p['verify']['ok'], p['verify']['failures_rank0'])
"
