set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "me_ or sr16 or inter or videocodec or closed_loop or motion" > gpurun_out/r04c_pytest_me.log 2>&1 || { tail -30 gpurun_out/r04c_pytest_me.log; exit 1; }
tail -2 gpurun_out/r04c_pytest_me.log
timeout -k 10 400 python -u tools/ab/ab_me.py ab/me_base.so ab/me_perm.so ab/me_ring.so --rounds 5 --oracle 2>&1 | tee gpurun_out/r04c_ab_me.log
