#!/usr/bin/env python3
"""Summarize rocprofv3 --kernel-trace/--stats CSVs into a markdown table
(calls, mean/min time, LDS bytes per workgroup, VGPRs, grid) for profiles/.

    python scripts/summarize_prof.py gpurun_out/prof_kern/kb > profiles/kernels.md
"""
import csv
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(pdcc::kern::DType\)(\d)", lambda m: ["f32", "f16", "bf16", "f64", "i8", "u8", "i32", "i64", "bool"][int(m.group(1))], name)
    name = re.sub(r"\(pdcc::kern::RedOp\)(\d)", lambda m: ["sum", "avg", "prod", "min", "max", "band", "bor", "bxor", "copy"][int(m.group(1))], name)
    name = name.replace("void ", "")
    name = re.sub(r"\(pdcc::[^)]*\)$", "", name)
    name = re.sub(r"\(.*", "", name) if not name.startswith("pdcc") else name
    return name[:110]


def main(prefix: str):
    stats = {}
    with open(prefix + "_kernel_stats.csv") as f:
        for r in csv.DictReader(f):
            stats[r["Name"]] = r
    trace = defaultdict(list)
    with open(prefix + "_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            trace[r["Kernel_Name"]].append(r)
    print(f"Source: `{os.path.basename(prefix)}_kernel_stats.csv` / `_kernel_trace.csv` (rocprofv3 --kernel-trace --stats)\n")
    print("| kernel | calls | mean us | min us | LDS B/WG | VGPR | SGPR | WG size | grid (WGs) |")
    print("|---|---|---|---|---|---|---|---|---|")
    rows = sorted(stats.values(), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows:
        name = r["Name"]
        if "pdcc" not in name and float(r["Percentage"]) < 2.0:
            continue
        t = trace.get(name, [{}])[0]
        wg = int(t.get("Workgroup_Size_X", 0) or 0)
        grid = int(t.get("Grid_Size_X", 0) or 0)
        print(
            f"| `{short(name)}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['MinNs'])/1e3:.1f} | "
            f"{t.get('LDS_Block_Size', '?')} | {t.get('VGPR_Count', '?')} | {t.get('SGPR_Count', '?')} | {wg} | "
            f"{grid // wg if wg else '?'} |"
        )


if __name__ == "__main__":
    main(sys.argv[1])
