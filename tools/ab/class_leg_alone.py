"""bench.py's class_api leg alone in a fresh process (no other legs before it), for comparison
with the same leg inside the full bench run:  python tools/ab/class_leg_alone.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

torch.cuda.set_device(0)
res = {}
bench.leg_class_api(None, torch.device("cuda", 0), res, None)
print(json.dumps({k: v for k, v in res["class_api"].items() if k != "note"}))
