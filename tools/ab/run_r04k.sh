# r04k: decode parse with 4 symbols per lane; emitter window flushed in 16-byte quads; the
# bench with the one-rank RCCL exchange (exit status and stderr kept)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/dec_zf.so ab/dec_p4.so --rounds 5 --legs symbols2image > gpurun_out/r04k_ab_dec.log 2>&1 || { tail -20 gpurun_out/r04k_ab_dec.log; exit 1; }
tail -4 gpurun_out/r04k_ab_dec.log
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/emit_pf2.so ab/emit_f4.so --rounds 5 --legs intra_symbols,symbols_hist > gpurun_out/r04k_ab_emit.log 2>&1 || { tail -20 gpurun_out/r04k_ab_emit.log; exit 1; }
tail -6 gpurun_out/r04k_ab_emit.log
timeout -k 10 900 python -u bench.py --rccl > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err; rc=$?
echo "bench rc=$rc"; tail -c 1500 gpurun_out/r04k_bench.err; [ $rc -eq 0 ] || exit $rc
python -c "
import json; d=json.load(open('gpurun_out/r04k_bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'verify', d['verify']['ok'], d['verify']['failures_rank0'])
for k in ('luma_only','image2symbols','zerorun','decode','inter','sharded','exchange','cfg2','class_api'):
    v=d.get(k); print(k, json.dumps(v)[:330] if v else None)"
