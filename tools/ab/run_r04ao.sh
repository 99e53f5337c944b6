# r04ao: per-chunk scans on the second stream (cur) vs on the caller's stream (prev, d500572) on
# one box: same-process timing of the pipelined legs, then bench.py legs with each library
# (the box's scratch copy of the tree gets prev's library for the second bench run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/prev.so ab/cur.so --rounds 9 --legs symbols_hist,zerorun_encode > gpurun_out/r04ao_ab.log 2>&1 || { tail -20 gpurun_out/r04ao_ab.log; exit 1; }
tail -5 gpurun_out/r04ao_ab.log
for v in cur prev; do
  cp ab/$v.so ivclab_amd/_lib/libivc.so
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --no-pmc > gpurun_out/r04ao_bench_$v.json 2> gpurun_out/r04ao_bench_$v.err || { tail -20 gpurun_out/r04ao_bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04ao_bench_$v.json'));print('$v','i2s',d['image2symbols']['ms'],'zr',d['zerorun']['ms'],'dec',d['decode']['ms'],'frac',d['roofline']['frac'])"
done
