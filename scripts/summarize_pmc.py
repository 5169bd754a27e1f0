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


def label(k):
    """(kernel label, source count) from a dispatch's kernel name; None for other kernels."""
    m = re.search(r"k1_reduce_(lds|stream|regs)<\(pdcc::kern::DType\)\d+, \(pdcc::kern::RedOp\)\d+, (\d+)", k)
    if m:
        return f"k1 {m.group(1)}", int(m.group(2))
    if "CUDAFunctor_add" in k or ("add" in k and "vectorized_elementwise" in k):
        return "torch.add", 2
    return None


def main(root):
    passes = {t: load(os.path.join(root, t)) for t in ("rd", "wr", "fetch", "write")}
    mib = int(os.environ.get("PDCC_PMC_MIB", "512"))
    print("# PMC byte reconciliation: K1 and torch.add on 512 MiB fp32 sources (above the 256 MiB MALL)\n")
    print("`scripts/pmc_passes.sh` (four rocprofv3 --pmc passes, one counter set each) over "
          "`scripts/pmc_k1_big.py`; MiB per dispatch. EA read MiB = 32 B x RDREQ_32B + 64 B x RDREQ_64B + "
          "128 B x RDREQ_128B (the raw TCC->EA requests by size); FETCH_SIZE is rocprof's derived counter, "
          "whose gfx950 formula counts 128-byte reads through TCC_BUBBLE.\n")
    print("| dispatch | kernel | nsrc | must read | RDREQ 32B / 64B / 128B (M) | EA read MiB | TCC_BUBBLE | "
          "FETCH_SIZE MiB | must write | WRREQ / WRREQ_64B (M) | WRITE_SIZE MiB |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for d in sorted(passes["rd"]):
        lab = label(passes["rd"][d].get("kernel", ""))
        if lab is None:
            continue
        name, nsrc = lab
        rd, wr = passes["rd"].get(d, {}), passes["wr"].get(d, {})
        r32, r64, r128 = (rd.get(f"TCC_EA0_RDREQ_{x}_sum", 0.0) for x in ("32B", "64B", "128B"))
        tot = rd.get("TCC_EA0_RDREQ_sum", 0.0)
        ea = (32 * r32 + 64 * r64 + 128 * r128 + 64 * max(0.0, tot - r32 - r64 - r128)) / MIB
        fetch = passes["fetch"].get(d, {}).get("FETCH_SIZE", 0.0) / 1024
        write = passes["write"].get(d, {}).get("WRITE_SIZE", 0.0) / 1024
        print(f"| {d} | {name} | {nsrc} | {nsrc * mib} | {r32 / 1e6:.2f} / {r64 / 1e6:.2f} / {r128 / 1e6:.2f} | "
              f"{ea:.1f} | {wr.get('TCC_BUBBLE_sum', 0.0):.0f} | {fetch:.1f} | {mib} | "
              f"{wr.get('TCC_EA0_WRREQ_sum', 0.0) / 1e6:.2f} / {wr.get('TCC_EA0_WRREQ_64B_sum', 0.0) / 1e6:.2f} | "
              f"{write:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc4")
