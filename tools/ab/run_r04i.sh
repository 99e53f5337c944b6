# r04i: emitter prefetch A/B (vector vs scalar loads of the next group's count/offset/flag),
# decode A/B (zf_count tile prefetch, DPP block-plane starts, rows stored from registers)
# with ablations (stores / parse skipped), the pinned-pool and symbol tests, the full bench
# (one-rank RCCL exchange), kernel times of the symbol legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/emit_head.so ab/emit_pf.so ab/emit_pf2.so --rounds 5 --legs intra_symbols,symbols_hist > gpurun_out/r04i_ab_emit.log 2>&1 || { tail -20 gpurun_out/r04i_ab_emit.log; exit 1; }
tail -6 gpurun_out/r04i_ab_emit.log
timeout -k 10 500 python -u tools/ab/ab_symbols.py ab/dec_a0.so ab/dec_zf.so ab/dec_zfdpp.so ab/dec_dir.so ab/dec_dirnt.so ab/dec_a1.so ab/dec_a2.so ab/dec_a3.so --rounds 4 --legs symbols2image > gpurun_out/r04i_ab_dec.log 2>&1 || { tail -20 gpurun_out/r04i_ab_dec.log; exit 1; }
tail -10 gpurun_out/r04i_ab_dec.log
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "pinned or tiny or pipeline or symbols or closed_loop" > gpurun_out/r04i_pytest.log 2>&1 || { tail -30 gpurun_out/r04i_pytest.log; exit 1; }
tail -1 gpurun_out/r04i_pytest.log
timeout -k 10 900 python bench.py --rccl > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err || { tail -20 gpurun_out/r04i_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r04i_bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'verify', d['verify']['ok'], d['verify']['failures_rank0'])
for k in ('luma_only','image2symbols','zerorun','decode','inter','sharded','exchange','cfg2','class_api'):
    v=d.get(k); print(k, json.dumps(v)[:330] if v else None)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04i_sym" -o run -- python tools/ab/ab_symbols.py ivclab_amd/_lib/libivc.so --rounds 2 --legs intra_symbols,symbols_hist,symbols2image,zerorun_encode > gpurun_out/r04i_prof_sym.log 2>&1 || { tail -20 gpurun_out/r04i_prof_sym.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_r04i_sym gpurun_out/r04i_sym_kernels.md "rocprofv3 --kernel-trace --stats -- python tools/ab/ab_symbols.py ivclab_amd/_lib/libivc.so --rounds 2 --legs intra_symbols,symbols_hist,symbols2image,zerorun_encode"
head -24 gpurun_out/r04i_sym_kernels.md
