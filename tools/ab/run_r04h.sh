# r04h: the c8 emitter A/B (tiles-per-row fix; outputs cleared per variant), the decode
# prefetch A/B on a real stream, then every GPU test and smoke with the in-tree build
# (two-block-row ME, c8 emitter, luma unpaced, host pipeline off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/emit_fused.so ab/emit_c8.so --rounds 5 --legs intra_symbols,symbols_hist 2>&1 | tee gpurun_out/r04h_ab_emit.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/dec_pf0w4.so ab/dec_pf5w3.so ab/dec_pf2w4.so --rounds 5 --legs symbols2image 2>&1 | tee gpurun_out/r04h_ab_dec.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04h_pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/r04h_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04h_smoke.log 2>&1 && echo smoke ok
