# r04z: round evidence on the final build (every GPU test, smoke, the bench with the driver's
# arguments, its kernel trace, the HBM traffic passes), then the bench once more with --rccl
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=r04z BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 1000 bash tools/round_evidence.sh > gpurun_out/r04z_evidence.log 2>&1; rc=$?; tail -c 800 gpurun_out/r04w_evidence.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --rccl --no-cpu --no-pmc > gpurun_out/r04z_bench_rccl.json 2> gpurun_out/r04z_bench_rccl.err || { tail -20 gpurun_out/r04z_bench_rccl.err; exit 1; }
echo rccl ok
