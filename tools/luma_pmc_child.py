"""Profiling child: the luma-only variant of the headline kernel (fused_encode_kernel<u8, f64,
C=1, OUT_LUMA>: 256 synthetic 4K luma frames -> [F, 270, 480, 64] int32 of the luminance
table plane) launched twice, unpaced (IVC_PACE_FIXED=0 is not needed: a fresh process runs the
first launches at the start rate).  Run under `rocprofv3 --pmc ...` (tools/gpu_pmc_child.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import ivclab_amd.device as D  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    F, H, W = int(os.environ.get("LUMA_FRAMES", "256")), 2160, 3840
    frames = bench.intra_frames(F, H, W, seed=3, dev=dev)
    table = PatchQuant(1.0).get_quantization_table()
    lum = torch.empty((F, H // 8, W // 8, 64), dtype=torch.int32, device=dev)
    for _ in range(2):
        D.intra_encode_luma(frames, table, lum)
    torch.cuda.synchronize()
    print("luma_pmc_child done")


if __name__ == "__main__":
    main()
