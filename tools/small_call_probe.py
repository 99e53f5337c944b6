"""The bench's small_call numbers alone (bench.small_call_us): the reference's per-block loop
calls through the drop-in classes and through NumPy, median per call."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ivclab_amd import DiscreteCosineTransform, PatchQuant  # noqa: E402
from oracle import ivc_oracle as O  # noqa: E402

rng = np.random.default_rng(1)
blk = rng.integers(0, 256, (8, 8)).astype(np.float64)
stk = rng.normal(0, 50, (3, 8, 8))
dct, pq = DiscreteCosineTransform(), PatchQuant(1.0)
assert np.array_equal(dct.transform(blk), O.dct_transform(blk))
assert np.array_equal(pq.quantize(stk), O.quantize(stk, 1.0))
from ivclab_amd import _native as N  # noqa: E402
for srv in (0, 1, 0):
    prev = N.set_tuning("tiny_server", srv)
    print(json.dumps(dict(bench.small_call_us(dct, pq, O, blk, stk), tiny_server=srv == 0)))
    N.set_tuning("tiny_server", prev)
