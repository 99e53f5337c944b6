# r04af: round evidence on the final sources (exec-masked zero-run emission writes) (every GPU test, smoke, bench with the driver's
# arguments, kernel trace, HBM traffic passes), the --rccl bench, the 2-rank gloo rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=r04af BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 1000 bash tools/round_evidence.sh > gpurun_out/r04af_evidence.log 2>&1; rc=$?; tail -c 600 gpurun_out/r04af_evidence.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --rccl --no-cpu --no-pmc > gpurun_out/r04af_bench_rccl.json 2> gpurun_out/r04af_bench_rccl.err || { tail -20 gpurun_out/r04af_bench_rccl.err; exit 1; }
echo rccl ok
timeout -k 10 700 bash tools/dist_rehearsal.sh > gpurun_out/r04af_dist.log 2>&1 || { tail -20 gpurun_out/r04af_dist.log; exit 1; }
echo dist ok
