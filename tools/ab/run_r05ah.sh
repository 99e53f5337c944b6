#!/bin/bash
# r05ah: race probe, many reps, current ME merge placement (mn) vs the round-4 one (mo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in mn mo mn mo; do
  timeout -k 10 300 python -u tools/race_probe.py --reps 150 --quiet --lib ab/$v.so >> gpurun_out/r05ah_$v.log 2>&1 || { tail -20 gpurun_out/r05ah_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r05ah_$v.log | tail -12
done
