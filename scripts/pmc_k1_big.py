#!/usr/bin/env python3
"""Fixed workload for the byte-reconciling PMC passes (scripts/pmc_passes.sh): K1 on 2 and 8
fp32 sources of 512 MiB each -- twice the 256 MiB Infinity Cache (MALL), so every byte
comes from HBM -- plus torch.add on the same 2 sources. Each kernel runs 3 times; the
expected bytes per dispatch are nsrc x 512 MiB read and 512 MiB written."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_collective_communication_amd import ops  # noqa: E402

MIB = int(os.environ.get("PDCC_PMC_MIB", "512"))


def main():
    dev = torch.device("cuda", 0)
    n = (MIB << 20) // 4
    srcs = [torch.rand(n, device=dev) for _ in range(8)]
    out = torch.empty(n, device=dev)
    for nsrc in (2, 8):
        for impl in ("lds_ntl", "stream_ntl"):
            for _ in range(3):
                ops.reduce_nway(srcs[:nsrc], out=out, impl=impl)
    for _ in range(3):
        torch.add(srcs[0], srcs[1], out=out)
    torch.cuda.synchronize()
    ok = torch.equal(ops.reduce_nway(srcs[:2], out=out), srcs[0] + srcs[1])
    print("pmc workload ok:", bool(ok), "MiB per source:", MIB)


if __name__ == "__main__":
    main()
