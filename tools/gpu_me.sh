#!/bin/bash
# ME iteration loop on the GPU box: ME/inter parity tests, then the inter bench leg under
# rocprofv3 --kernel-trace --stats (summary in gpurun_out/me_kernels.md).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -k "me_ or motion or inter or device_api" -p no:cacheprovider > gpurun_out/pytest_me.log 2>&1 || { tail -30 gpurun_out/pytest_me.log; exit 1; }
tail -1 gpurun_out/pytest_me.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_me" -o run -- python bench.py --no-intra --no-cpu ${BENCH_ARGS} > gpurun_out/bench_me.json 2> gpurun_out/bench_me.err || { tail -20 gpurun_out/bench_me.err; exit 1; }
python -c "import json; print(json.load(open('gpurun_out/bench_me.json'))['inter'])"
python tools/prof_summary.py gpurun_out/prof_me gpurun_out/me_kernels.md "rocprofv3 --kernel-trace --stats -- python bench.py --no-intra --no-cpu ${BENCH_ARGS}"
find gpurun_out/prof_me -name "*kernel_trace.csv" -delete
grep "ivc::" gpurun_out/me_kernels.md
