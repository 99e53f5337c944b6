# r04u: symbols2image pipelined over K chunks of tiles (zf_count/scan/locate of chunk j+1 on the
# caller's stream overlapping the decode of chunk j-1 on a second stream), K = 8, 16, 32, 64;
# the decode tests in-tree (K = 16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/s2i_k8.so ab/s2i_k16.so ab/s2i_k32.so ab/s2i_k64.so --rounds 7 --legs symbols2image > gpurun_out/r04u_ab_s2i.log 2>&1 || { tail -20 gpurun_out/r04u_ab_s2i.log; exit 1; }
tail -7 gpurun_out/r04u_ab_s2i.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "symbols2image or decode or zerorun or closed_loop or intracodec" > gpurun_out/r04u_pytest.log 2>&1 || { tail -30 gpurun_out/r04u_pytest.log; exit 1; }
tail -1 gpurun_out/r04u_pytest.log
