#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a profiling child:
#   CHILD=tools/sym_pmc_child.py PMC_GROUPS=tools/pmc_groups_me.txt OUTDIR=pmc_sym bash tools/gpu_pmc_child.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/${OUTDIR:-pmc_child}"
mkdir -p "$OUT"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- python $CHILD > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done < "${PMC_GROUPS:-tools/pmc_groups_me.txt}"
python tools/pmc_reduce.py "gpurun_out/${OUTDIR:-pmc_child}"
