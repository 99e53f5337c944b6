# r04f: symbols A/B (fixed histogram bins), class-API breakdown (+ kernel / copy trace), and
# PMC of the new ME kernel and of the fit emission pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/sym_base.so ab/sym_fit.so ab/sym_mask.so --rounds 5 --legs intra_symbols,symbols_hist 2>&1 | tee gpurun_out/r04f_ab_sym.log
timeout -k 10 300 python -u tools/class_api_breakdown.py --json gpurun_out/r04f_class_api.json 2>&1 | tee gpurun_out/r04f_class_api.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04f_cls" -o run -- python tools/class_api_breakdown.py > gpurun_out/r04f_class_prof.log 2>&1 || { tail -20 gpurun_out/r04f_class_prof.log; exit 1; }
find gpurun_out/prof_r04f_cls -name "*_trace.csv" -delete
CHILD=tools/me_pmc_child.py ME_NO_F64=1 PMC_GROUPS=tools/pmc_groups_me.txt OUTDIR=pmc_r04f_me timeout -k 10 600 bash tools/gpu_pmc_child.sh > gpurun_out/r04f_pmc_me.log 2>&1 || { tail -20 gpurun_out/r04f_pmc_me.log; exit 1; }
CHILD=tools/sym_pmc_child.py SYM_DECODE=0 PMC_GROUPS=tools/pmc_groups_sym3.txt OUTDIR=pmc_r04f_sym timeout -k 10 600 bash tools/gpu_pmc_child.sh > gpurun_out/r04f_pmc_sym.log 2>&1 || { tail -20 gpurun_out/r04f_pmc_sym.log; exit 1; }
echo done
