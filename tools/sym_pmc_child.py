"""Profiling child: the cfg3 entropy stages alone — ZeroRunCoder.encode of the zig-zag
coefficients (zw_count / scan / zw_emit) and the fused pixels -> symbols path (fused encoder
OUT_COUNT / scan / OUT_SYMBOLS, then OUT_SYMH with the histogram), then
the decode leg (intra_decode_image of the coefficients, symbols2image of the stream), once each on 256 (SYM_FRAMES) 4K frames.  Run under
`rocprofv3 --pmc ...`."""
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
    F = int(os.environ.get("SYM_FRAMES", "256"))
    H, W = 2160, 3840
    frames = bench.intra_frames(F, H, W, seed=3, dev=dev).view(F, H, W, 1)
    table = PatchQuant(1.0).get_quantization_table()
    out = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
    D.intra_encode(frames, table, out, zigzag=True)
    nblk = out.numel() // 64
    offs = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
    probe = torch.empty(1, dtype=torch.int32, device=dev)
    D.zerorun_encode(out.view(nblk, 64), offs, probe)
    nsym = int(offs[-1].item())
    sym = torch.empty(nsym, dtype=torch.int32, device=dev)
    D.zerorun_encode(out.view(nblk, 64), offs, sym)
    nsd = torch.zeros(1, dtype=torch.int64, device=dev)
    D.intra_symbols(frames, table, sym, nsd)
    # the bench's form: the emission pass also accumulates the stream's histogram (OUT_SYMH)
    hist = torch.zeros(bench.HIST_BINS + 2, dtype=torch.int64, device=dev)
    D.intra_symbols(frames, table, sym, nsd, hist=hist, hist_lo=bench.HIST_LO - 1)
    torch.cuda.synchronize()
    if os.environ.get("SYM_DECODE", "1") == "1":
        # the decode leg: coefficients -> RGB image, and the fused symbols -> RGB image
        del frames
        img = torch.empty((F, H, W, 3), dtype=torch.float64, device=dev)
        D.intra_decode_image(out, table, img, unzigzag=True, to_rgb=True)
        err = torch.zeros(3, dtype=torch.int64, device=dev)
        D.symbols2image(sym, 3, table, img, err, to_rgb=True)
        torch.cuda.synchronize()
    print("sym_pmc_child done", nsym)


if __name__ == "__main__":
    main()
