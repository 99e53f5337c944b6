# r04am: symbols2image with the per-chunk scan, locate and group range on the second stream
# (ahead of the decode they feed) instead of between the caller's EOB passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/s16.so ab/s2ia.so --rounds 9 --legs symbols2image > gpurun_out/r04am_ab_s2i.log 2>&1 || { tail -20 gpurun_out/r04am_ab_s2i.log; exit 1; }
tail -4 gpurun_out/r04am_ab_s2i.log
