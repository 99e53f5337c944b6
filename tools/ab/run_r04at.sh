# r04at: decode chunk count on the bench's 256 frames with the 16 K-tile minimum (K = 32 default,
# 16, 24, 48), same-process timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/dk32.so ab/dk16.so ab/dk24.so ab/dk48.so --rounds 7 --legs symbols2image > gpurun_out/r04at_ab_dec.log 2>&1 || { tail -20 gpurun_out/r04at_ab_dec.log; exit 1; }
tail -5 gpurun_out/r04at_ab_dec.log
