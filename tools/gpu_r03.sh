#!/bin/bash
# Round-3 development call: the parity tests selected by $TESTS (pytest -k expression, all
# GPU tests when empty), then the bench with the driver's own arguments.  Each GPU step has
# its own time limit; a failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider ${TESTS:+-k "$TESTS"} > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_$TAG.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  python - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
rl = d["roofline"]; sp = rl.get("store_pace", {})
print("value", d["value"], "frac", rl["frac"], "kernel_ms", rl["kernel_ms"], "traffic_x", rl.get("traffic_vs_algorithmic"))
print("pace", {k: v for k, v in sp.items() if not k.startswith("trace")})
for k in ("decode", "inter", "image2symbols", "zerorun", "exchange", "sharded", "verify"):
    if k in d:
        print(k, json.dumps(d[k])[:400])
PY
fi
