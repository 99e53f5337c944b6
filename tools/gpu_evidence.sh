set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r01f.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r01f.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r01f.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r01f.log 2>&1 || { tail -20 gpurun_out/smoke_r01f.log; exit 1; }
tail -1 gpurun_out/smoke_r01f.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r01f.json 2> gpurun_out/bench_r01f.err || { tail -20 gpurun_out/bench_r01f.err; exit 1; }
cat gpurun_out/bench_r01f.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r01f" -o run -- python bench.py --no-cpu > gpurun_out/prof_r01f.log 2>&1 || { tail -20 gpurun_out/prof_r01f.log; exit 1; }
echo prof ok
