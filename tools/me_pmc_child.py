"""Profiling child: the cfg4 motion search alone (1080p x 300 u8, +-16, exact SSD: the
matrix-core me_mfma16_kernel), twice, then (unless ME_NO_F64=1) the float64 NumPy-semantics
search on 60 frames once.  Run under `rocprofv3 --pmc ...` (tools/gpu_pmc_child.sh); prints nothing timed."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import ivclab_amd.device as D  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    F = int(os.environ.get("ME_FRAMES", "300"))
    seq = bench.inter_frames(F, 1080, 1920, seed=4, dev=dev)
    mv = torch.empty((F - 1, 135, 240), dtype=torch.int64, device=dev)
    for _ in range(2):
        D.motion_estimate(seq[:-1], seq[1:], 16, mv, exact_u8=True)
    if os.environ.get("ME_NO_F64") != "1":
        y = bench.luma_f64(seq[:60]).contiguous()
        mvf = torch.empty((59, 135, 240), dtype=torch.int64, device=dev)
        D.motion_estimate(y[:-1], y[1:], 16, mvf)
    torch.cuda.synchronize()
    print("me_pmc_child done")


if __name__ == "__main__":
    main()
