# r04v: zero-run encode pipelined over K chunks of groups (count of chunk j+1 beside the
# emission of chunk j on a second stream), K = 1, 8, 16, 32; zero-run and decode tests in-tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/zrp_k1.so ab/zrp_k8.so ab/zrp_k16.so ab/zrp_k32.so --rounds 7 --legs zerorun_encode > gpurun_out/r04v_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04v_ab_zr.log; exit 1; }
tail -6 gpurun_out/r04v_ab_zr.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "symbols2image or decode or zerorun or closed_loop or intracodec" > gpurun_out/r04v_pytest.log 2>&1 || { tail -30 gpurun_out/r04v_pytest.log; exit 1; }
tail -1 gpurun_out/r04v_pytest.log
