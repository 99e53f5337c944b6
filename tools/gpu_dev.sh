#!/bin/bash
# Development loop on the GPU box: GPU parity tests (all, or $TESTS), then the default bench
# line (optionally $BENCH_ARGS).  Outputs under gpurun_out/.  Each GPU step has its own time
# limit; a failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-dev}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_$TAG.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; cat gpurun_out/bench_$TAG.json; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi
