#!/bin/bash
# r06ac: zero-run encode with the sparse int8 hand-off (IVC_ZC_SPARSE=1: masks + packed
# nonzeros per group) — the zero-run parity tests on the in-tree build (sparse on), then a
# same-process A/B against the dense hand-off, outputs compared.  Correct (129 passed) but
# 10.64 -> 11.99 ms (profiles/r06ac_ab_zerorun_sparse.log): the packing and unpacking cost more
# issue and a wave of occupancy than the ~7 GB it saves; the variant was removed after this run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workload.py -q -x -m gpu -k "zerorun or zero_run or symbols or intra" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ac_pytest_zr.log 2>&1 || { tail -40 gpurun_out/r06ac_pytest_zr.log; exit 1; }
tail -2 gpurun_out/r06ac_pytest_zr.log
timeout -k 10 600 python tools/ab/ab_zr.py ab/base.so ab/sparse.so --rounds 5 > gpurun_out/r06ac_ab_zerorun_sparse.log 2>&1 || { tail -20 gpurun_out/r06ac_ab_zerorun_sparse.log; exit 1; }
cat gpurun_out/r06ac_ab_zerorun_sparse.log
