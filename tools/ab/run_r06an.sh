#!/bin/bash
# r06an: cfg2 repeated launches checked launch by launch (tools/cfg2_repro.py), plain and under
# rocprofv3 --pmc WRITE_SIZE (where one evidence run's bench verify failed cfg2 frames 0 / 63)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cfg2_repro.py > gpurun_out/r06an_cfg2_plain.log 2>&1; echo "plain rc=$?" >> gpurun_out/r06an_cfg2_plain.log
tail -3 gpurun_out/r06an_cfg2_plain.log
timeout -s KILL 250 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r06an_pmc" -o run -- python -u tools/cfg2_repro.py > gpurun_out/r06an_cfg2_pmc.log 2>&1; echo "pmc rc=$?" >> gpurun_out/r06an_cfg2_pmc.log
grep -v "^[EW]2026" gpurun_out/r06an_cfg2_pmc.log | tail -8
