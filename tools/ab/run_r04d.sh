# r04d: ME (permuted blocks, ring operand) and the fit emission path: parity tests with the
# in-tree build, then same-process A/Bs of the built variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "me_ or sr16 or inter or videocodec or closed_loop or motion or symbol or zerorun or intra or rd_curve" > gpurun_out/r04d_pytest.log 2>&1 || { tail -30 gpurun_out/r04d_pytest.log; exit 1; }
tail -2 gpurun_out/r04d_pytest.log
timeout -k 10 300 python -u tools/ab/ab_me.py ab/me_base.so ab/me_perm.so ab/sym_fit.so --rounds 5 --oracle 2>&1 | tee gpurun_out/r04d_ab_me.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/sym_base.so ab/sym_fit.so ab/sym_mask.so --rounds 5 --legs intra_symbols,symbols_hist 2>&1 | tee gpurun_out/r04d_ab_sym.log
