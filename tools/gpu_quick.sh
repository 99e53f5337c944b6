#!/bin/bash
# Development loop on the GPU box: all GPU parity tests, then the bench (no CPU legs)
# under rocprofv3 --kernel-trace --stats; prints the bench line and the ivc:: kernel rows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_q" -o run -- python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -20 gpurun_out/bench_q.err; exit 1; }
cat gpurun_out/bench_q.json
python tools/prof_summary.py gpurun_out/prof_q gpurun_out/q_kernels.md "rocprofv3 --kernel-trace --stats -- python bench.py --no-cpu ${BENCH_ARGS}"
find gpurun_out/prof_q -name "*kernel_trace.csv" -delete
grep "ivc::" gpurun_out/q_kernels.md
