#!/usr/bin/env python3
"""Reconcile the PMC passes of scripts/pmc_passes.sh into one markdown table.

Per dispatch of scripts/pmc_k1_big.py (3 runs per kernel; the last of each is shown):
raw TCC->EA read requests by size (32 / 64 / 128 B), the byte total they add up to,
TCC_BUBBLE (what rocprof's gfx950 FETCH_SIZE formula takes as the 128-byte count),
rocprof's derived FETCH_SIZE / WRITE_SIZE, and the bytes the kernel must move
(nsrc x S read, S written).

    python scripts/summarize_pmc.py gpurun_out/pmc4 > profiles/r4/pmc_k1_reconciled.md
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

MIB = 1 << 20


def load(pass_dir):
    """{dispatch id: {"kernel": name, counter: value}} from one pass's counter_collection csv."""
    out = defaultdict(dict)
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                d = int(r.get("Dispatch_Id") or r.get("Dispatch-Id") or 0)
                out[d]["kernel"] = r.get("Kernel_Name", "")
                name = r.get("Counter_Name", "")
                out[d][name] = out[d].get(name, 0.0) + float(r.get("Counter_Value", 0) or 0)
    return out


def short(k):
    if "k1_" in k:
        m = re.search(r"(k1_\w+)<[^,]*,[^,]*,\s*(\d)", k)
        return m.group(1) if m else k[:40]
    if "add" in k.lower() or "elementwise" in k.lower():
        return "torch.add"
    return k[:40]


def main(root):
    passes = {t: load(os.path.join(root, t)) for t in ("rd", "wr", "fetch", "write")}
    ids = sorted(set().union(*[set(p) for p in passes.values()]))
    mib = int(os.environ.get("PDCC_PMC_MIB", "512"))
    # dispatch order of pmc_k1_big.py: (2 src: lds_ntl x3, stream_ntl x3), (8 src: same), torch.add x3
    expect = [(2, "k1 lds_ntl")] * 3 + [(2, "k1 stream_ntl")] * 3 + [(8, "k1 lds_ntl")] * 3 + \
             [(8, "k1 stream_ntl")] * 3 + [(2, "torch.add")] * 3
    big = [d for d in ids if "reduce" in passes["rd"].get(d, {}).get("kernel", "") or
           "add" in passes["rd"].get(d, {}).get("kernel", "").lower() or "elementwise" in
           passes["rd"].get(d, {}).get("kernel", "").lower()]
    print("# PMC byte reconciliation: K1 and torch.add on 512 MiB fp32 sources (above the 256 MiB MALL)\n")
    print("`scripts/pmc_passes.sh` (four rocprofv3 --pmc passes, one counter set each) over "
          "`scripts/pmc_k1_big.py`. MiB per dispatch; requests x their size = EA read bytes.\n")
    print("| dispatch | kernel | nsrc | must read | RDREQ 32B/64B/128B (M) | EA read MiB | TCC_BUBBLE (M) "
          "| FETCH_SIZE MiB | must write | WRREQ (M) 64B (M) | WRITE_SIZE MiB |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    rows = [d for d in ids if d in passes["rd"]][-len(expect):] if len(big) < len(expect) else big[-len(expect):]
    for d, (nsrc, label) in zip(rows, expect):
        rd, wr = passes["rd"].get(d, {}), passes["wr"].get(d, {})
        r32, r64, r128 = (rd.get(f"TCC_EA0_RDREQ_{s}_sum", 0.0) for s in ("32B", "64B", "128B"))
        tot = rd.get("TCC_EA0_RDREQ_sum", 0.0)
        ea = (32 * r32 + 64 * r64 + 128 * r128 + 64 * max(0.0, tot - r32 - r64 - r128)) / MIB
        fetch = passes["fetch"].get(d, {}).get("FETCH_SIZE", 0.0) / 1024
        write = passes["write"].get(d, {}).get("WRITE_SIZE", 0.0) / 1024
        print(f"| {d} | {label} | {nsrc} | {nsrc * mib} | {r32 / 1e6:.2f} / {r64 / 1e6:.2f} / {r128 / 1e6:.2f} | "
              f"{ea:.1f} | {wr.get('TCC_BUBBLE_sum', 0.0) / 1e6:.2f} | {fetch:.1f} | {mib} | "
              f"{wr.get('TCC_EA0_WRREQ_sum', 0.0) / 1e6:.2f} {wr.get('TCC_EA0_WRREQ_64B_sum', 0.0) / 1e6:.2f} | "
              f"{write:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc4")
