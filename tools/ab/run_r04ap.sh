# r04ap: chunk counts with the per-chunk scans on the second stream: zero-run K = 16 / 24 / 32 / 48,
# pixels -> symbols K = 12 / 16 / 20 (same-process timing)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/zk32.so ab/zk16.so ab/zk24.so ab/zk48.so --rounds 7 --legs zerorun_encode > gpurun_out/r04ap_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04ap_ab_zr.log; exit 1; }
tail -5 gpurun_out/r04ap_ab_zr.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/zk32.so ab/sk12.so ab/sk20.so --rounds 7 --legs symbols_hist > gpurun_out/r04ap_ab_sym.log 2>&1 || { tail -20 gpurun_out/r04ap_ab_sym.log; exit 1; }
tail -4 gpurun_out/r04ap_ab_sym.log
