# r04e: symbols A/B on real frames (ab_symbols.py buffer fix) and the class-API breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/sym_base.so ab/sym_fit.so ab/sym_mask.so --rounds 5 --legs intra_symbols,symbols_hist 2>&1 | tee gpurun_out/r04e_ab_sym.log
timeout -k 10 300 python -u tools/class_api_breakdown.py --json gpurun_out/r04e_class_api.json 2>&1 | tee gpurun_out/r04e_class_api.log
