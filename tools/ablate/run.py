"""Phase ablation of the fused intra kernel on the bench workload (256 x 4K luma frames).
Builds tools/ablate/ablate.hip into /tmp, then times each skip mask in interleaved rounds.
    python tools/ablate/run.py [frames]
bits: 1 row DCT, 2 column DCT, 4 quantisation, 8 LDS transpose, 16 stores, 32 loads."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
VARIANT = os.environ.get("ABL_DEFS", "")   # e.g. "-DIVC_STORE_AUX=2 -DIVC_LOAD_AUX=2"
so = "/tmp/ivc_ablate%s.so" % abs(hash(VARIANT))
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                "-ffp-contract=off", *VARIANT.split(), "-o", so, os.path.join(HERE, "ablate.hip"),
                os.path.join(ROOT, "ivclab_amd", "csrc", "ivc_entropy.hip")], check=True)
print("variant:", VARIANT or "(default)")
sys.path.insert(0, ROOT)
import ivclab_amd._native as N  # noqa: E402  (shares torch's HIP runtime)
N.load_library()
L = ctypes.CDLL(so)
L.diag_intra_u8.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                            ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
H, W = 2160, 3840
dev = torch.device("cuda:0")
import bench  # noqa: E402
img = (bench.intra_frames(F, H, W, seed=3, dev=dev) if os.environ.get("ABL_DATA", "bench") == "bench"
       else torch.randint(0, 256, (F, H, W), dtype=torch.uint8, device=dev))
out = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
from ivclab_amd import PatchQuant  # noqa: E402
t = N.table_arg(PatchQuant(1.0).get_quantization_table())
modes = {}
for ng in [int(x) for x in os.environ.get("ABL_NG", "1,2,4,8").split(",")]:
    modes[f"ng{ng} full"] = (0, ng)
    modes[f"ng{ng} mem-only"] = (15, ng)
    modes[f"ng{ng} no-load"] = (32, ng)
    modes[f"ng{ng} no-store"] = (16, ng)
    modes[f"ng{ng} loads-only"] = (31, ng)
    modes[f"ng{ng} stores-only"] = (47, ng)
res = {k: [] for k in modes}
res["torch fill_ (same buffer)"] = []
ms = ctypes.c_float()


def fill_ms():
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out.fill_(0)
    s_.record()
    for _ in range(3):
        out.fill_(0)
    e_.record()
    torch.cuda.synchronize()
    return s_.elapsed_time(e_) / 3


for rnd in range(5):
    res["torch fill_ (same buffer)"].append(fill_ms())
    for k, (m, ng) in modes.items():
        rc = L.diag_intra_u8(img.data_ptr(), F, H, W, t.ctypes.data, out.data_ptr(), m, ng, 3, ctypes.byref(ms))
        assert rc == 0, rc
        res[k].append(ms.value)
bytes_ = F * H * W * 13
for k, v in res.items():
    med = float(np.median(v))
    print(f"{k:26s} median {med:8.3f} ms  min {min(v):8.3f}  ({bytes_ / med / 1e6:8.1f} GB/s algorithmic, "
          f"{out.numel() * 4 / med / 1e6:8.1f} GB/s of output)")
