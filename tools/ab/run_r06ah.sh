#!/bin/bash
# r06ah: PMC of the round-6 ±16 ME kernel (me_mfma16x2_kernel after the energy-phase change),
# the counter groups of tools/pmc_groups_me.txt, one rocprofv3 --pmc pass each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
ME_NO_F64=1 CHILD="tools/me_pmc_child.py" PMC_GROUPS=tools/pmc_groups_me.txt OUTDIR=r06ah_pmc_me timeout -k 10 600 bash tools/gpu_pmc_child.sh > gpurun_out/r06ah_pmc_me.log 2>&1 || { tail -20 gpurun_out/r06ah_pmc_me.log; exit 1; }
cat gpurun_out/r06ah_pmc_me.log
find gpurun_out/r06ah_pmc_me -name "*.json" | head
