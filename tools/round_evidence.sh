#!/bin/bash
# One GPU call that produces the round's evidence: GPU parity tests, smoke, the default
# bench line, a rocprofv3 --kernel-trace --stats run of the same bench, and the HBM
# FETCH_SIZE/WRITE_SIZE passes of the intra kernel (separate --pmc runs).  Outputs under
# gpurun_out/; the caller copies what is judged into profiles/.  Every GPU step has its own
# time limit and a failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
  echo smoke ok
  # the cfg5 step repeated against an unchunked single-stream run, bitwise (the r05 LDS race)
  timeout -k 10 300 python -u tools/race_probe.py --reps 300 --quiet > gpurun_out/race_probe_$TAG.log 2>&1 || { tail -20 gpurun_out/race_probe_$TAG.log; exit 1; }
  timeout -k 10 300 python -u tools/race_probe.py --mode intra --reps 60 --quiet >> gpurun_out/race_probe_$TAG.log 2>&1 || { tail -20 gpurun_out/race_probe_$TAG.log; exit 1; }
  grep "runs differ" gpurun_out/race_probe_$TAG.log
fi
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python bench.py --no-cpu --no-pmc ${BENCH_ARGS} > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_$TAG gpurun_out/${TAG}_bench_kernels.md "rocprofv3 --kernel-trace --stats -- python bench.py --no-cpu --no-pmc ${BENCH_ARGS}" || true
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
head -8 gpurun_out/${TAG}_bench_kernels.md
if [ -z "$SKIP_PMC" ]; then
  PMC_GROUPS=tools/pmc_groups_hbm.txt CMD="python bench.py --steps 3 --warmup 1 --no-inter --no-cpu --no-pmc" \
    timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
  python tools/pmc_traffic.py gpurun_out/pmc/summary.json 256 2160 3840 gpurun_out/pmc_intra_latest.json
fi
