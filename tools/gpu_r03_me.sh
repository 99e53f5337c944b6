#!/bin/bash
# Matrix-core +-16 search (IVC_ME_MFMA=1) vs the dot4 tiled search: the sr = 16 parity tests
# with the MFMA kernel selected, then the cfg4 inter leg alternately with each kernel on the
# same box (separate processes: the switch is read once per process).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || IVC_ME_MFMA=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "${ME_TESTS:-me_ or sr16 or inter or videocodec or smoke}" > gpurun_out/pytest_me.log 2>&1 || { tail -40 gpurun_out/pytest_me.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/pytest_me.log
INTER_ONLY="--no-intra --no-symbols --no-f64 --no-class-api --no-sharded --no-cpu --no-pmc --no-luma --inter-steps 5"
for mode in ${MODES:-0 1 0 1}; do            # m or m:var (IVC_ME_VAR: ivc_me_mfma.hip)
  m=${mode%%:*}; var=0; [[ $mode == *:* ]] && var=${mode#*:}
  IVC_ME_MFMA=$m IVC_ME_VAR=$var timeout -k 10 300 python bench.py $INTER_ONLY > gpurun_out/me_$m.json 2> gpurun_out/me_$m.err || { tail -5 gpurun_out/me_$m.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/me_$m.json')); i=d['inter']; r=i['roofline']
print('mfma=$m var=$var inter ms', i['ms_per_step'], 'search ms', r['kernel_ms'], 'dot4-frac', r['frac'], 'verify', d['verify']['ok'])"
done
# PROF=1: per-kernel durations (kernel trace) and the ME PMC groups over the search child, with
# the kernel IVC_ME_MFMA selects (default 1)
if [ -n "$PROF" ]; then
  export IVC_ME_MFMA=${PROF_MFMA:-1} ME_FRAMES=${ME_FRAMES:-300}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_me$IVC_ME_MFMA" -o run -- python tools/me_pmc_child.py > gpurun_out/prof_me.log 2>&1 || { tail -20 gpurun_out/prof_me.log; exit 1; }
  python tools/prof_summary.py gpurun_out/prof_me$IVC_ME_MFMA gpurun_out/prof_me$IVC_ME_MFMA.md "IVC_ME_MFMA=$IVC_ME_MFMA rocprofv3 --kernel-trace --stats -- python tools/me_pmc_child.py" | grep -E "me_" | cut -c1-150
  find gpurun_out/prof_me$IVC_ME_MFMA -name "*kernel_trace.csv" -delete
  CHILD=tools/me_pmc_child.py OUTDIR=pmc_me$IVC_ME_MFMA bash tools/gpu_pmc_child.sh > gpurun_out/pmc_me.log 2>&1 || { tail -20 gpurun_out/pmc_me.log; exit 1; }
  echo "pmc summary: gpurun_out/pmc_me$IVC_ME_MFMA/summary.json"
fi
