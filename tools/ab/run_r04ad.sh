# r04ad: zero-run emitter writes exec-masked (no dummy words) vs the dummy-word form: same-process
# timing of the zero-run encode, then the emitter's LDS counters for each variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/zcx0.so ab/zcx1.so ab/zcx2.so ab/zcx3.so --rounds 7 --legs zerorun_encode > gpurun_out/r04ad_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04ad_ab_zr.log; exit 1; }
tail -6 gpurun_out/r04ad_ab_zr.log
for v in 0 1 2 3; do
  CHILD="tools/ab/ab_symbols.py ab/zcx$v.so --rounds 1 --frames 64 --legs zerorun_encode" PMC_GROUPS=tools/pmc_groups_zc.txt OUTDIR=r04ad_pmc_zcx$v timeout -k 10 200 bash tools/gpu_pmc_child.sh > gpurun_out/r04ad_pmc_zcx$v.log 2>&1 || { tail -20 gpurun_out/r04ad_pmc_zcx$v.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04ad_pmc_zcx$v/summary.json'));print($v,{k:{c:round(x['mean']) for c,x in v.items()} for k,v in d.items() if 'zc_emit' in k})"
done
