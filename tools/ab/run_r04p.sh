# r04p: the zero-run count pass with the int8 hand-off: non-temporal c8 stores, 2 groups per
# wave-iteration (fewer VGPRs); the emitter histogram's out-of-range symbols handled after the
# flush loop; the 2-rank gloo rehearsal of bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/zr_base.so ab/zr_zc2.so ab/zr_zc_nt.so ab/zr_zc_g2.so ab/zr_zc_ntg2.so --rounds 7 --legs zerorun_encode > gpurun_out/r04p_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04p_ab_zr.log; exit 1; }
tail -7 gpurun_out/r04p_ab_zr.log
timeout -k 10 300 python -u tools/ab/ab_symbols.py ab/emit_tl0.so ab/emit_tl.so --rounds 7 --legs symbols_hist > gpurun_out/r04p_ab_emit.log 2>&1 || { tail -20 gpurun_out/r04p_ab_emit.log; exit 1; }
tail -4 gpurun_out/r04p_ab_emit.log
# the multi-rank bench path (2 gloo ranks on cuda:0) with the one-JSON-line stdout
timeout -k 10 700 bash tools/dist_rehearsal.sh > gpurun_out/r04p_dist.log 2>&1; rc=$?; tail -c 600 gpurun_out/r04p_dist.log; [ $rc -eq 0 ] || exit $rc
python -c "
import json; t=open('gpurun_out/dist2.json').read(); lines=[l for l in t.splitlines() if l.strip()]
print('stdout lines', len(lines)); d=json.loads(lines[0]); print('n_gpus', d['n_gpus'], 'value', d['value'], 'verify', d['verify']['ok'])"
