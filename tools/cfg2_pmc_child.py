"""Profiling child: cfg2's kernel (fused_encode_kernel<u8, f64, C=3, ZZ>: 64 synthetic 1080p RGB
frames -> [64, 135, 240, 3, 64] int32) launched 3 times from the library given as argv[1]
(default: the product build).  Run under `rocprofv3 --pmc ...` (tools/gpu_pmc_child.sh with
CHILD="tools/cfg2_pmc_child.py ab/x.so")."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import ivclab_amd._native as N  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    L = N.load_library()
    if len(sys.argv) > 1:
        L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
        for name, (a, r) in N._SIGS.items():
            fn = getattr(L, name, None)
            if fn is not None:
                fn.argtypes, fn.restype = a, r
    F, H, W = int(os.environ.get("CFG2_FRAMES", "64")), 1080, 1920
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    frames = torch.randint(0, 256, (F, H, W, 3), device=dev, generator=g, dtype=torch.uint8)
    out = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    t = N.table_arg(PatchQuant(1.0).get_quantization_table())
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        assert L.ivc_intra_encode_dev(frames.data_ptr(), 1, F, H, W, 3, N.ptr(t), 10, 1,
                                      out.data_ptr(), None, 0, 0, s) == 0
    torch.cuda.synchronize()
    print("cfg2_pmc_child done")


if __name__ == "__main__":
    main()
