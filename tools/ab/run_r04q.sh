# r04q: emission slots as one mbcnt chain (fill folded in) in both emitters; zero-run and
# zf_count with wave-contiguous quarters and a DPP count (decode); zero-run and symbol tests with the in-tree build (int8 hand-off + non-temporal c8, chained slots)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/emit_tl0.so ab/emit_sc.so ab/cnt_mm.so ab/emit_fs.so --rounds 7 --legs intra_symbols,symbols_hist > gpurun_out/r04q_ab_emit.log 2>&1 || { tail -20 gpurun_out/r04q_ab_emit.log; exit 1; }
tail -6 gpurun_out/r04q_ab_emit.log
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/zr_base.so ab/zr_zc_nt.so ab/zr_zc3.so ab/cnt_mm.so --rounds 7 --legs zerorun_encode > gpurun_out/r04q_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04q_ab_zr.log; exit 1; }
tail -5 gpurun_out/r04q_ab_zr.log
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/dec_zf0.so ab/dec_zfc.so ab/dec_clip.so --rounds 7 --legs symbols2image > gpurun_out/r04q_ab_dec.log 2>&1 || { tail -20 gpurun_out/r04q_ab_dec.log; exit 1; }
tail -4 gpurun_out/r04q_ab_dec.log
# (the full GPU test run is part of the evidence below)

# round evidence with the in-tree build: every GPU test, smoke, the bench with the driver's
# arguments, its kernel trace, the HBM traffic passes
TAG=r04q BENCH_ARGS="--steps 20 --warmup 5" SKIP_TESTS= timeout -k 10 1000 bash tools/round_evidence.sh > gpurun_out/r04q_evidence.log 2>&1; rc=$?; tail -c 1500 gpurun_out/r04q_evidence.log; exit $rc
