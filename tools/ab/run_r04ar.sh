# r04ar: chunk-size minimums (new) on a 64-frame batch against no pipelining (sk1) and on the
# bench's 256 frames against the fixed counts (sk16); decode chunk counts on 64 frames
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/sk1.so ab/new.so --frames 64 --rounds 9 --legs symbols_hist,zerorun_encode > gpurun_out/r04ar_ab64.log 2>&1 || { tail -20 gpurun_out/r04ar_ab64.log; exit 1; }
tail -5 gpurun_out/r04ar_ab64.log
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/new.so ab/d1.so ab/d8.so ab/d16.so --frames 64 --rounds 9 --legs symbols2image > gpurun_out/r04ar_ab64_dec.log 2>&1 || { tail -20 gpurun_out/r04ar_ab64_dec.log; exit 1; }
tail -5 gpurun_out/r04ar_ab64_dec.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/sk16.so ab/new.so --rounds 7 --legs symbols_hist,zerorun_encode > gpurun_out/r04ar_ab256.log 2>&1 || { tail -20 gpurun_out/r04ar_ab256.log; exit 1; }
tail -5 gpurun_out/r04ar_ab256.log
