# r04g: same-process A/Bs (ME software pipelining and the two-block-row tile; the c8 symbol
# emitter; zero-run lane emit; decode prefetch), class-API breakdown (pipeline on/off,
# zero-copy tiny calls), luma-only PMC, then the GPU tests of the touched paths
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_me.py ab/me_swp0r4.so ab/me_swp1r2.so ab/me_swp1r10.so ab/me_2row.so --rounds 5 --oracle 2>&1 | tee gpurun_out/r04g_ab_me.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/emit_fused.so ab/emit_c8.so --rounds 5 --legs intra_symbols,symbols_hist 2>&1 | tee gpurun_out/r04g_ab_emit.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/zw_old.so ab/zw_lane.so --rounds 5 --legs zerorun_encode 2>&1 | tee gpurun_out/r04g_ab_zw.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/dec_pf0w4.so ab/dec_pf5w3.so ab/dec_pf2w4.so --rounds 5 --legs symbols2image 2>&1 | tee gpurun_out/r04g_ab_dec.log
timeout -k 10 300 python -u tools/class_api_breakdown.py --json gpurun_out/r04g_class_api.json 2>&1 | tee gpurun_out/r04g_class_api.log
IVC_PACE_GBPS=0 CHILD=tools/luma_pmc_child.py PMC_GROUPS=tools/pmc_groups_luma.txt OUTDIR=pmc_r04g_luma timeout -k 10 600 bash tools/gpu_pmc_child.sh > gpurun_out/r04g_pmc_luma.log 2>&1 || { tail -20 gpurun_out/r04g_pmc_luma.log; exit 1; }
echo luma pmc done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 200 --timeout-method thread -p no:cacheprovider -k "dct or quant or zigzag or tiny or pipeline or dropin or ch3 or symbol or decode or me_ or sr16 or zerorun or rd_curve or closed_loop" > gpurun_out/r04g_pytest.log 2>&1; tail -15 gpurun_out/r04g_pytest.log
