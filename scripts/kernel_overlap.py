#!/usr/bin/env python3
"""Per-rank durations and cross-rank overlap of one kernel in a rocprofv3 kernel trace.

Ranks sharing one GPU each launch their own copy of a gated IPC kernel; the device phase
trace (scripts/ipc_phase_trace.py) only stamps block 0. This reads the whole-dispatch
start/end of every rank's launches of the kernels whose name matches PATTERN and pairs
the i-th launch of each process: per rank the median duration, and per pair the start skew
(how long the first rank's kernel ran before its peer's started) and the union span.

    python scripts/kernel_overlap.py gpurun_out/prof_zc/zc_kernel_trace.csv k_ipc_reduce
"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict


def main(path, pattern):
    rx = re.compile(pattern)
    per_pid = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if rx.search(r.get("Kernel_Name", "")):
                pid = r.get("Process_Id") or r.get("Pid") or "0"
                per_pid[pid].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                     int(r.get("Grid_Size_X", 0) or 0) // max(1, int(r.get("Workgroup_Size_X", 1) or 1))))
    out = {"kernel_pattern": pattern, "ranks": {}}
    for pid, v in sorted(per_pid.items()):
        v.sort()
        d = [(e - s) / 1e3 for s, e, _ in v]
        out["ranks"][pid] = {"launches": len(v), "median_us": round(statistics.median(d), 1),
                             "min_us": round(min(d), 1), "max_us": round(max(d), 1), "workgroups": v[0][2]}
    pids = sorted(per_pid)
    if len(pids) >= 2:
        n = min(len(per_pid[p]) for p in pids)
        skew, span = [], []
        for i in range(n):
            ls = [per_pid[p][i] for p in pids]
            skew.append((max(s for s, _, _ in ls) - min(s for s, _, _ in ls)) / 1e3)
            span.append((max(e for _, e, _ in ls) - min(s for s, _, _ in ls)) / 1e3)
        out["pairs"] = n
        out["start_skew_median_us"] = round(statistics.median(skew), 1)
        out["union_span_median_us"] = round(statistics.median(span), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_ipc_reduce")
