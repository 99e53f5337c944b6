# r04ai: pixels -> symbols chunk count around K = 16 (12, 16, 20, 24; same-process timing), and the
# same with a one-rank RCCL group created first (its streams take hardware queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/symk12.so ab/symk16.so ab/symk20.so ab/symk24.so --rounds 7 --legs intra_symbols,symbols_hist > gpurun_out/r04ai_ab_sym.log 2>&1 || { tail -20 gpurun_out/r04ai_ab_sym.log; exit 1; }
tail -10 gpurun_out/r04ai_ab_sym.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/symk12.so ab/symk16.so ab/symk20.so ab/symk24.so --rounds 5 --rccl --legs symbols_hist > gpurun_out/r04ai_ab_sym_rccl.log 2>&1 || { tail -20 gpurun_out/r04ai_ab_sym_rccl.log; exit 1; }
tail -6 gpurun_out/r04ai_ab_sym_rccl.log
