"""cfg2 (1920x1080 RGB, C = 3 fused encode) repeated the way bench.py's leg runs it — 200
one-frame launches, then 240 launches of a 64-frame batch — and every launch's output checked:
each one-frame launch against the oracle's frame 0, each batch launch against the first batch
launch (digest), and frames 0 / 63 of the last against the oracle.  Prints the launches and
elements that differ.  Run plain and under rocprofv3 --pmc (tools/ab/run_r06an.sh)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ivclab_amd.device as D  # noqa: E402
from ivclab_amd import PatchQuant  # noqa: E402
from ivclab_amd import _native as N  # noqa: E402
from oracle import ivc_oracle as O  # noqa: E402

dev = torch.device("cuda:0")
F, H, W = 64, 1080, 1920
g = torch.Generator(device=dev)
g.manual_seed(1)
frames = torch.randint(0, 256, (F, H, W, 3), device=dev, generator=g, dtype=torch.uint8)
out = torch.empty((F, H // 8, W // 8, 3, 64), dtype=torch.int32, device=dev)
table = N.table_arg(PatchQuant(1.0).get_quantization_table())
want0 = torch.from_numpy(O.intra_encode(frames[0].cpu().numpy(), 1.0, zigzag=True).reshape(out[0].shape))
want63 = torch.from_numpy(O.intra_encode(frames[F - 1].cpu().numpy(), 1.0, zigzag=True).reshape(out[0].shape))
bad = 0
for i in range(200):
    out[0].fill_(-7)
    D.intra_encode(frames[:1], table, out[:1], zigzag=True)
    torch.cuda.synchronize()
    d = int((out[0].cpu() != want0).sum())
    if d:
        bad += 1
        print(f"one-frame launch {i}: {d} elements differ", flush=True)
ref = None
for i in range(240):
    out.fill_(-7)
    D.intra_encode(frames, table, out, zigzag=True)
    torch.cuda.synchronize()
    s = (out.view(-1).to(torch.int64) * (torch.arange(out.numel(), device=dev) % 7919 + 1)).sum().item()
    if ref is None:
        ref = s
        d0 = int((out[0].cpu() != want0).sum())
        d63 = int((out[F - 1].cpu() != want63).sum())
        print(f"batch launch 0: frame 0 {d0} / frame 63 {d63} elements differ from the oracle", flush=True)
        bad += (d0 > 0) + (d63 > 0)
    elif s != ref:
        bad += 1
        nd = int((out.cpu() != out.cpu()).sum())
        print(f"batch launch {i}: digest differs", flush=True)
d0 = int((out[0].cpu() != want0).sum())
d63 = int((out[F - 1].cpu() != want63).sum())
print(f"last batch: frame 0 {d0} / frame 63 {d63} elements differ; {bad} bad launches", flush=True)
sys.exit(1 if bad or d0 or d63 else 0)
