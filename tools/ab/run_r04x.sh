# r04x: inter encode pipelined over K chunks of frame pairs (ME of chunk j+1 on the caller's
# stream beside the residual encode of chunk j on the second stream), K = 1, 4, 8, 16; the inter
# tests with K forced to 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_inter.py ab/inter_k1.so ab/inter_k4.so ab/inter_k8.so ab/inter_k16.so --rounds 5 > gpurun_out/r04x_ab_inter.log 2>&1 || { tail -20 gpurun_out/r04x_ab_inter.log; exit 1; }
tail -10 gpurun_out/r04x_ab_inter.log
IVC_INTER_FORCE_CHUNKS=3 timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "inter or closed_loop or video or sharded" > gpurun_out/r04x_pytest.log 2>&1 || { tail -30 gpurun_out/r04x_pytest.log; exit 1; }
tail -1 gpurun_out/r04x_pytest.log
