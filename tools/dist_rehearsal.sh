#!/bin/bash
# Rehearse bench.py's multi-rank path on a one-GPU box: 2 ranks on cuda:0 over gloo
# (RCCL needs one GPU per rank), small sizes.  The driver's N>1 runs use nccl.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
IVC_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  --frames 16 --inter-frames 20 --sharded-frames 12 --no-cpu > gpurun_out/dist2.json 2> gpurun_out/dist2.err
rc=$?
cat gpurun_out/dist2.json; tail -5 gpurun_out/dist2.err
exit $rc
