#!/bin/bash
# Round-2 re-entry GPU call: the full GPU parity suite at HEAD, then PMC passes (one counter
# group per rocprofv3 run) over the cfg4 motion search alone (outputs gpurun_out/pmc_me/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_me"
mkdir -p "$OUT"
CMD="python tools/me_pmc_child.py"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- $CMD > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done < tools/pmc_groups_me.txt
python tools/pmc_reduce.py gpurun_out/pmc_me
