#!/bin/bash
# GPU-box check used during development: parity tests, smoke, a short bench, a rocprof
# kernel-trace of the bench.  Every GPU step has its own time limit; a step that faults or
# times out ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-5}
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=40 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps $STEPS --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python bench.py --steps $STEPS --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/prof.log 2>&1; rc=$?
  tail -3 gpurun_out/prof.log; find gpurun_out/prof -name "*stats*"; exit $rc
fi
