# r04l: decode A/B (4-symbol parse, integer-table dequantiser + one 1/16 scaling), then every
# GPU test with the in-tree build (parse4 + DQ_INT default), smoke, and the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/dec_zf.so ab/dec_p4.so ab/dec_dq.so ab/dec_dqp4.so --rounds 5 --legs symbols2image > gpurun_out/r04l_ab_dec.log 2>&1 || { tail -20 gpurun_out/r04l_ab_dec.log; exit 1; }
tail -6 gpurun_out/r04l_ab_dec.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04l_pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/r04l_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04l_smoke.log 2>&1 && echo smoke ok
timeout -k 10 900 python -u bench.py --rccl > gpurun_out/r04l_bench.json 2> gpurun_out/r04l_bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -c 1500 gpurun_out/r04l_bench.err; exit $rc; }
python -c "
import json; d=json.loads(open('gpurun_out/r04l_bench.json').read())
print('value', d['value'], 'frac', d['roofline']['frac'], 'verify', d['verify']['ok'], d['verify']['failures_rank0'])
for k in ('luma_only','image2symbols','zerorun','decode','inter','sharded','exchange','cfg2','class_api'):
    v=d.get(k); print(k, json.dumps(v)[:300] if v else None)"
