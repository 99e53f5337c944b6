# r04aj: kernel traces of the pipelined pixels -> symbols call with K = 16 and K = 24 (the
# K >= 24 slowdown of r04ai), one round each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for k in 16 24; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r04aj_k$k" -o run -- python tools/ab/ab_symbols.py ab/symk$k.so --rounds 1 --legs symbols_hist > gpurun_out/r04aj_k$k.log 2>&1 || { tail -20 gpurun_out/r04aj_k$k.log; exit 1; }
  tail -2 gpurun_out/r04aj_k$k.log
done
