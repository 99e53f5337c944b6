# r04r: final build — PMC of the symbol kernels (5 passes), then the round evidence (every GPU
# test, smoke, bench with the driver's arguments, kernel trace, HBM traffic passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CHILD=tools/sym_pmc_child.py PMC_GROUPS=tools/pmc_groups_sym.txt OUTDIR=pmc_r04r_sym timeout -k 10 600 bash tools/gpu_pmc_child.sh > gpurun_out/r04r_pmc_sym.log 2>&1 || { tail -20 gpurun_out/r04r_pmc_sym.log; exit 1; }
echo pmc done
TAG=r04r BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 1000 bash tools/round_evidence.sh > gpurun_out/r04r_evidence.log 2>&1; rc=$?; tail -c 1200 gpurun_out/r04r_evidence.log; exit $rc
