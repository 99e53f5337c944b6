# r04ag: the class-API chain three ways on one box — the breakdown tool, bench.py's class_api leg
# alone in a fresh process, and the same leg inside the full bench run (per-rep times)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/class_api_breakdown.py --json gpurun_out/r04ag_class_api.json > gpurun_out/r04ag_breakdown.log 2>&1 || { tail -20 gpurun_out/r04ag_breakdown.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04ag_class_api.json'));print({k:(v['chain_ms'],v['chain_nopipe_ms']) for k,v in d.items() if 'chain_ms' in v})"
timeout -k 10 300 python tools/ab/class_leg_alone.py > gpurun_out/r04ag_leg_alone.json 2> gpurun_out/r04ag_leg_alone.err || { tail -20 gpurun_out/r04ag_leg_alone.err; exit 1; }
cut -c1-600 gpurun_out/r04ag_leg_alone.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04ag_bench.json 2> gpurun_out/r04ag_bench.err || { tail -20 gpurun_out/r04ag_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04ag_bench.json'))['class_api'];print({k:v for k,v in d.items() if k!='note'})"
