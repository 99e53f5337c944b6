#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace/--stats only alongside)
# over the intra bench; outputs under gpurun_out/pmc/<group>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
CMD=${CMD:-"python bench.py --steps 3 --warmup 1 --no-inter --no-cpu --no-pmc"}
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- $CMD > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done < "${PMC_GROUPS:-tools/pmc_groups.txt}"
python tools/pmc_reduce.py gpurun_out/pmc
