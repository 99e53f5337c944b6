# r04ae: exec-masked emission writes in both emitters (zero-run: the new default; pixels -> symbols: IVC_EMIT_EXEC) vs the dummy-word form:
# timing, the emitter's LDS counters for both, then the zero-run / decode GPU tests
# (the ab/*.so variants were built at commit ceee3cb with -DIVC_ZC_EXEC=0 / -DIVC_EMIT_EXEC=0,1; the
# dropped forms were removed afterwards: zero-run keeps the exec-masked writes, pixels -> symbols the dummy words)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/zcx0.so ab/zcxn.so --rounds 9 --legs zerorun_encode > gpurun_out/r04ae_ab_zr.log 2>&1 || { tail -20 gpurun_out/r04ae_ab_zr.log; exit 1; }
tail -4 gpurun_out/r04ae_ab_zr.log
for v in 0 n; do
  CHILD="tools/ab/ab_symbols.py ab/zcx$v.so --rounds 1 --legs zerorun_encode" PMC_GROUPS=tools/pmc_groups_zc.txt OUTDIR=r04ae_pmc_zcx$v timeout -k 10 200 bash tools/gpu_pmc_child.sh > gpurun_out/r04ae_pmc_zcx$v.log 2>&1 || { tail -20 gpurun_out/r04ae_pmc_zcx$v.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04ae_pmc_zcx$v/summary.json'));k=d['ivc::zc_emit_kernel'];print('$v',{c:round(x['mean']) for c,x in k.items()},'conflicts/LDS instr',round(k['SQ_LDS_BANK_CONFLICT']['mean']/k['SQ_INSTS_LDS']['mean'],3))"
done
timeout -k 10 400 python -u tools/ab/ab_symbols.py ab/emx0.so ab/emx1.so --rounds 9 --legs intra_symbols,symbols_hist > gpurun_out/r04ae_ab_sym.log 2>&1 || { tail -20 gpurun_out/r04ae_ab_sym.log; exit 1; }
tail -6 gpurun_out/r04ae_ab_sym.log
for v in 0 1; do
  CHILD="tools/ab/ab_symbols.py ab/emx$v.so --rounds 1 --legs symbols_hist" PMC_GROUPS=tools/pmc_groups_zc.txt OUTDIR=r04ae_pmc_emx$v timeout -k 10 200 bash tools/gpu_pmc_child.sh > gpurun_out/r04ae_pmc_emx$v.log 2>&1 || { tail -20 gpurun_out/r04ae_pmc_emx$v.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04ae_pmc_emx$v/summary.json'));[print('$v',n,{c:round(x['mean']) for c,x in k.items()},'conflicts/LDS instr',round(k['SQ_LDS_BANK_CONFLICT']['mean']/k['SQ_INSTS_LDS']['mean'],3)) for n,k in d.items()]"
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "zerorun or symbols2image or decode or intracodec" > gpurun_out/r04ae_pytest.log 2>&1 || { tail -30 gpurun_out/r04ae_pytest.log; exit 1; }
tail -1 gpurun_out/r04ae_pytest.log
