# r04o: zero-run encode with the int8 hand-off written by zw_count (register layout, bpermute
# transpose in the emitter) against the two-pass int32 path; zero-run tests in-tree; kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/zr_base.so ab/zr_zc2.so --rounds 7 --legs zerorun_encode > gpurun_out/r04o_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04o_ab_zr.log; exit 1; }
tail -4 gpurun_out/r04o_ab_zr.log
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "zerorun or closed_loop" > gpurun_out/r04o_pytest.log 2>&1 || { tail -30 gpurun_out/r04o_pytest.log; exit 1; }
tail -1 gpurun_out/r04o_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04o" -o run -- python tools/ab/ab_symbols.py ivclab_amd/_lib/libivc.so --rounds 2 --legs zerorun_encode,symbols2image,symbols_hist > gpurun_out/r04o_prof.log 2>&1 || { tail -20 gpurun_out/r04o_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_r04o gpurun_out/r04o_kernels.md "rocprofv3 --kernel-trace --stats -- python tools/ab/ab_symbols.py ivclab_amd/_lib/libivc.so --rounds 2 --legs zerorun_encode,symbols2image,symbols_hist"
grep -E "zw_|zc_|sym_|zf_" gpurun_out/r04o_kernels.md
