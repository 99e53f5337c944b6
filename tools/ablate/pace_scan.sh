for p in 0 6000 6600; do echo "== pace $p"; IVC_PACE_GBPS=$p ABL_NG=2 timeout -k 10 200 python tools/ablate/run.py 2>&1 | grep -v amdgpu.ids | grep "ng2\|fill" || exit 1; done
