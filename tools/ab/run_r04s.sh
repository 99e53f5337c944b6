# r04s: non-temporal stores of the pixels -> symbols hand-off (count pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/c8_base.so ab/c8_nt.so --rounds 9 --legs intra_symbols,symbols_hist > gpurun_out/r04s_ab_c8.log 2>&1 || { tail -20 gpurun_out/r04s_ab_c8.log; exit 1; }
tail -6 gpurun_out/r04s_ab_c8.log
