"""Condense a rocprofv3 --kernel-trace --stats output directory into profiles/<name>.md:
per-kernel calls / average / min / max duration and the resources of each ivc:: kernel.
    python tools/prof_summary.py gpurun_out/prof profiles/r01_bench_kernels.md "<command>"
"""
import csv
import glob
import os
import sys


def main(d, out, cmd=""):
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    res = {}
    for r in csv.DictReader(open(trace)):
        res.setdefault(r["Kernel_Name"], r)
    lines = [f"# rocprofv3 kernel summary", "", f"command: `{cmd}`", "",
             "| kernel | calls | avg ms | min ms | max ms | % time | VGPR | SGPR | LDS B | grid x wg |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats)):
        n = r["Name"]
        short = n.split("(")[0].replace("void ", "")
        if len(short) > 90:
            short = short[:87] + "..."
        t = res.get(n, {})
        lines.append(f"| `{short}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.4f} | "
                     f"{float(r['MinNs'])/1e6:.4f} | {float(r['MaxNs'])/1e6:.4f} | {float(r['Percentage']):.2f} | "
                     f"{t.get('VGPR_Count','')} | {t.get('SGPR_Count','')} | {t.get('LDS_Block_Size','')} | "
                     f"{t.get('Grid_Size_X','')} x {t.get('Workgroup_Size_X','')} |")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:16]))


if __name__ == "__main__":
    main(*sys.argv[1:])
