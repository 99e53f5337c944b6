# r04g: GPU tests of the touched paths, class-API breakdown (pipeline on/off, zero-copy tiny
# calls), ME software-pipelining A/B, decode prefetch A/B, zero-run emit A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "dct or quant or zigzag or tiny or pipeline or dropin or ch3 or symbols2image or decode or me_ or sr16 or zerorun" > gpurun_out/r04g_pytest.log 2>&1 || { tail -30 gpurun_out/r04g_pytest.log; exit 1; }
tail -2 gpurun_out/r04g_pytest.log
timeout -k 10 300 python -u tools/class_api_breakdown.py --json gpurun_out/r04g_class_api.json 2>&1 | tee gpurun_out/r04g_class_api.log
timeout -k 10 400 python -u tools/ab/ab_me.py ab/me_swp0r4.so ab/me_swp1r2.so ab/me_swp1r4.so ab/me_swp1r10.so --rounds 5 2>&1 | tee gpurun_out/r04g_ab_me.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/zw_old.so ab/zw_lane.so --rounds 5 --legs zerorun_encode 2>&1 | tee gpurun_out/r04g_ab_zw.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/dec_pf0w4.so ab/dec_pf5w3.so ab/dec_pf2w4.so ab/dec_pf3w4.so --rounds 5 --legs symbols2image 2>&1 | tee gpurun_out/r04g_ab_dec.log
echo done
