# r04y: pipelined symbols2image with each chunk's decode grid at 8/8, 7/8, 6/8 of the resident
# grid (room for the next chunk's EOB pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/s2ig_8.so ab/s2ig_7.so ab/s2ig_6.so --rounds 7 --legs symbols2image > gpurun_out/r04y_ab_s2i.log 2>&1 || { tail -20 gpurun_out/r04y_ab_s2i.log; exit 1; }
tail -5 gpurun_out/r04y_ab_s2i.log
