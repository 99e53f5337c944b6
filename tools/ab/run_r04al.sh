# r04al: the pipelined calls' per-chunk scans on the second stream (ahead of their emitter)
# instead of the caller's stream (between the count passes): pixels -> symbols at K = 16 / 24 /
# 32 and the zero-run encode (K = 32), same-process timing, outputs compared
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/s16.so ab/s16a.so ab/s24a.so ab/s32a.so --rounds 7 --legs intra_symbols,symbols_hist > gpurun_out/r04al_ab_sym.log 2>&1 || { tail -20 gpurun_out/r04al_ab_sym.log; exit 1; }
tail -10 gpurun_out/r04al_ab_sym.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/s16.so ab/s16a.so --rounds 9 --legs zerorun_encode > gpurun_out/r04al_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04al_ab_zr.log; exit 1; }
tail -4 gpurun_out/r04al_ab_zr.log
