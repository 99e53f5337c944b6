# r04ah: pixels -> symbols with the count pass and the emitter pipelined over K chunks of frames
# (K = 1, 8, 16, 32; same-process timing), then the symbol GPU tests in-tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "intra_symbols or intracodec or zerorun" > gpurun_out/r04ah_pytest.log 2>&1 || { tail -30 gpurun_out/r04ah_pytest.log; exit 1; }
tail -1 gpurun_out/r04ah_pytest.log
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/symk1.so ab/symk8.so ab/symk16.so ab/symk32.so --rounds 7 --legs intra_symbols,symbols_hist > gpurun_out/r04ah_ab_sym.log 2>&1 || { tail -20 gpurun_out/r04ah_ab_sym.log; exit 1; }
tail -10 gpurun_out/r04ah_ab_sym.log
