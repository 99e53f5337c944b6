# r04aq: pipelined calls on a 64-frame batch (a quarter of the bench's): is the slowdown seen
# at many chunks a matter of the chunk count or of the chunk size?  Variants: symbols / zero-run
# chunks 1/1, 4/8, 8/16, 16/32 (defaults)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/sk1.so ab/sk4.so ab/sk8.so ab/sk16.so --frames 64 --rounds 9 --legs symbols_hist,zerorun_encode > gpurun_out/r04aq_ab.log 2>&1 || { tail -20 gpurun_out/r04aq_ab.log; exit 1; }
tail -10 gpurun_out/r04aq_ab.log
