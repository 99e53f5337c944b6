ABL_DATA=bench timeout -k 10 300 python tools/ablate/run.py 2>&1 | grep -v amdgpu.ids || exit 1
ABL_DATA=noise timeout -k 10 300 python tools/ablate/run.py 2>&1 | grep -v amdgpu.ids || exit 1
