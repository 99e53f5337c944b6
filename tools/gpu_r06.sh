#!/bin/bash
# Round-6 GPU call: GPU parity tests (optional), then the default bench line.  Every GPU step has
# its own time limit and a failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider $TESTS > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_$TAG.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_$TAG.json').read());print(json.dumps(d['legs']))"
fi
