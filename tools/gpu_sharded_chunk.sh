#!/bin/bash
# A/B of the cfg5 (8K x 120, frame-sharded) bench step: pairs per inter_encode chunk and the
# workgroups per CU of the side-stream histograms.  Each run prints ms/step and the histogram
# checksum (must agree across runs).  Outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "histogram" > gpurun_out/sc_pytest.log 2>&1 || { tail -30 gpurun_out/sc_pytest.log; exit 1; }
tail -1 gpurun_out/sc_pytest.log
for cfg in "0 4" "8 4" "8 1" "8 2" "4 1" "16 1" "0 4" "8 1" "8 2"; do
  set -- $cfg
  tag=c$1_w$2
  timeout -k 10 300 python bench.py --no-intra --no-inter --no-cpu --sharded-steps 5 \
    --sharded-chunk $1 --sharded-hist-wg $2 > gpurun_out/sc_$tag.json 2> gpurun_out/sc_$tag.err \
    || { tail -20 gpurun_out/sc_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sc_$tag.json'))['sharded'];print('$tag',d['ms_per_step'],d['exchange']['hist_checksum'],d['exchange']['symbols'])"
done
