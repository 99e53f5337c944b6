# r04t: zf_count with a bounds-test-free path for whole tiles and one popcount per quad
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/zf_head.so ab/zf_full.so --rounds 9 --legs symbols2image > gpurun_out/r04t_ab_zf.log 2>&1 || { tail -20 gpurun_out/r04t_ab_zf.log; exit 1; }
tail -4 gpurun_out/r04t_ab_zf.log
