"""Reduce rocprofv3 --pmc CSV outputs (gpurun_out/pmc/g*/...counter_collection.csv) to a
per-kernel summary of the ivc:: kernels: mean counter value per dispatch.  Deletes the raw
per-dispatch CSVs afterwards (they include every torch data-generation kernel)."""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def main(root="gpurun_out/pmc", keep=False):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            n = r.get("Kernel_Name", "")
            if "ivc::" not in n:
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = n
        for (d, c), v in per.items():
            acc[names[d].split("(")[0].replace("void ", "")][c].append(v)
    out = {k: {c: {"mean": sum(v) / len(v), "n": len(v)} for c, v in cs.items()} for k, cs in acc.items()}
    with open(os.path.join(root, "summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    if not keep:
        for g in glob.glob(os.path.join(root, "g*")):
            if os.path.isdir(g):
                shutil.rmtree(g)
    for k, cs in out.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:40s} {v['mean']:.6g}  (n={v['n']})")


if __name__ == "__main__":
    main(*sys.argv[1:])
