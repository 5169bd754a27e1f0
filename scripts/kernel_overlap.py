#!/usr/bin/env python3
"""Per-rank durations and cross-rank overlap of one kernel in rocprofv3 kernel traces.

Ranks sharing one GPU each launch their own copy of a gated IPC kernel; the device phase
trace (scripts/ipc_phase_trace.py) stamps inside the kernel. This reads the whole-dispatch
start/end of every rank's launches of the kernels whose name matches PATTERN (one trace
file per process: rocprofv3 -o name_%pid%), keeps the launches at the largest grid, and
pairs the i-th launch of each rank: per rank the median duration, per pair the start skew
(how long the first rank's kernel ran before its peer's started) and the union span.

    python scripts/kernel_overlap.py k_ipc_reduce gpurun_out/prof_zc2/zc_*_kernel_trace.csv
"""
import csv
import json
import re
import statistics
import sys


def main(pattern, paths):
    rx = re.compile(pattern)
    per_rank = {}
    for path in paths:
        rows = []
        with open(path) as f:
            for r in csv.DictReader(f):
                if rx.search(r.get("Kernel_Name", "")):
                    wgs = int(r.get("Grid_Size_X", 0) or 0) // max(1, int(r.get("Workgroup_Size_X", 1) or 1))
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), wgs))
        if rows:
            big = max(w for _, _, w in rows)
            per_rank[path] = sorted(x for x in rows if x[2] == big)
    out = {"kernel_pattern": pattern, "ranks": {}}
    for path, v in per_rank.items():
        d = [(e - s) / 1e3 for s, e, _ in v]
        out["ranks"][path.rsplit("/", 1)[-1]] = {"launches": len(v), "workgroups": v[0][2],
                                                 "median_us": round(statistics.median(d), 1),
                                                 "min_us": round(min(d), 1), "max_us": round(max(d), 1)}
    keys = list(per_rank)
    if len(keys) >= 2:
        n = min(len(per_rank[k]) for k in keys)
        skew, span = [], []
        for i in range(n):
            ls = [per_rank[k][i] for k in keys]
            skew.append((max(s for s, _, _ in ls) - min(s for s, _, _ in ls)) / 1e3)
            span.append((max(e for _, e, _ in ls) - min(s for s, _, _ in ls)) / 1e3)
        out["pairs"] = n
        out["start_skew_median_us"] = round(statistics.median(skew), 1)
        out["union_span_median_us"] = round(statistics.median(span), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
