#!/bin/bash
# Kernel-trace the inter chain of each A/B library at 1080p x 300 and 8K x 24
# (per-kernel averages in gpurun_out/me_prof_<shape>.md).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for shape in 300x1080x1920 24x4320x7680; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$shape" -o run -- python tools/ab/ab_intra.py ${AB_LIBS} --frames 1 --rounds 2 --reps 2 --inter --inter-shape $shape > gpurun_out/me_prof_$shape.log 2>&1 || { tail -20 gpurun_out/me_prof_$shape.log; exit 1; }
  python tools/prof_summary.py gpurun_out/prof_$shape gpurun_out/me_prof_$shape.md "ab_intra --inter-shape $shape"
  find gpurun_out/prof_$shape -name "*kernel_trace.csv" -delete
  grep -E "me_|inter|fused_encode_kernel<unsigned char, unsigned char" gpurun_out/me_prof_$shape.md | cut -c1-140
done
