#!/bin/bash
# Round-2 first GPU call: the new workload-size parity tests, then the full GPU suite,
# then the VALU rate microbenchmark (f64 add/mul issue rates for the f64 ME roofline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_workload.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_workload.log 2>&1 || { tail -40 gpurun_out/pytest_workload.log; exit 1; }
tail -8 gpurun_out/pytest_workload.log
hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_rates tools/ubench/valu_rates.hip && timeout -k 10 60 /tmp/valu_rates > gpurun_out/valu_rates.txt 2>&1 || { cat gpurun_out/valu_rates.txt; exit 1; }
cat gpurun_out/valu_rates.txt
