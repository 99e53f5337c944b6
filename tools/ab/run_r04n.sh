# r04n: zero-run encode through the int8 hand-off (zc_count / zc_emit) against the two-pass
# int32 path; the zero-run tests with the hand-off in-tree; PMC of the symbol kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/zr_base.so ab/zr_zc.so --rounds 5 --legs zerorun_encode > gpurun_out/r04n_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04n_ab_zr.log; exit 1; }
tail -4 gpurun_out/r04n_ab_zr.log
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "zerorun or closed_loop or symbols" > gpurun_out/r04n_pytest.log 2>&1 || { tail -30 gpurun_out/r04n_pytest.log; exit 1; }
tail -1 gpurun_out/r04n_pytest.log
bash tools/ab/run_r04m.sh
