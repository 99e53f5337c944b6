#!/bin/bash
# The cfg3 entropy legs alone (zero-run encode, pixels -> symbols, the Huffman-table exchange,
# symbols -> image decode): the bench legs with verify, then (PROF=1) a kernel trace of the same
# run and (PMC=1) the symbol-stage PMC groups over tools/sym_pmc_child.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$TESTS" ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "$TESTS" > gpurun_out/pytest_sym.log 2>&1 || { tail -40 gpurun_out/pytest_sym.log; exit 1; }; tail -1 gpurun_out/pytest_sym.log; }
SYM_ONLY="--no-inter --no-f64 --no-class-api --no-sharded --no-cpu --no-pmc --no-luma --steps 3 --warmup 2"
timeout -k 10 400 python bench.py $SYM_ONLY > gpurun_out/sym.json 2> gpurun_out/sym.err || { tail -20 gpurun_out/sym.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/sym.json"))
print("image2symbols ms", d["image2symbols"]["ms"], "zerorun ms", d["zerorun"]["ms"],
      "exchange ms", d["exchange"]["ms"], "verify", d["verify"]["ok"])
dc = d.get("decode", {})
print("decode ms", dc.get("ms"), "frac", dc.get("roofline", {}).get("frac"),
      "coefficients_to_image ms", dc.get("coefficients_to_image", {}).get("kernel_ms"))
PY
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sym" -o run -- python bench.py $SYM_ONLY --no-verify > gpurun_out/prof_sym.log 2>&1 || { tail -20 gpurun_out/prof_sym.log; exit 1; }
  python tools/prof_summary.py gpurun_out/prof_sym gpurun_out/prof_sym.md "rocprofv3 --kernel-trace --stats -- python bench.py $SYM_ONLY --no-verify" | grep -E "zw_|zr_|zf_|fused|histogram|minmax|decode|scan" | cut -c1-150
  find gpurun_out/prof_sym -name "*kernel_trace.csv" -delete
fi
if [ -n "$PMC" ]; then
  CHILD=tools/sym_pmc_child.py PMC_GROUPS=tools/pmc_groups_sym.txt OUTDIR=pmc_sym bash tools/gpu_pmc_child.sh > gpurun_out/pmc_sym.log 2>&1 || { tail -20 gpurun_out/pmc_sym.log; exit 1; }
  echo "pmc summary: gpurun_out/pmc_sym/summary.json"
fi
