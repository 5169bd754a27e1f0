#!/usr/bin/env python3
"""Small fixed workload for rocprofv3 --pmc runs (scripts/profile.sh pmc):
K1 reduce_nway (LDS-DMA, register, LDS-DMA with non-temporal stores, streaming with
non-temporal stores / loads and stores) on 2 and 8 fp32 sources of
64 MiB, K2 multi_copy of 16 x 4 MiB, and torch.add as the HBM reference.
Each kernel runs 3 times, so per-dispatch counters (FETCH_SIZE, WRITE_SIZE,
LDS bank conflicts) can be read straight off the counter CSV."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_collective_communication_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = (64 << 20) // 4
    srcs = [torch.rand(n, device=dev) for _ in range(8)]
    out = torch.empty(n, device=dev)
    for nsrc in (2, 8):
        for variant in ("lds", "regs", "lds_nt", "stream_nt", "stream_ntl"):
            for _ in range(3):
                ops.reduce_nway(srcs[:nsrc], out=out, op="sum", impl=variant)
    for _ in range(3):
        torch.add(srcs[0], srcs[1], out=out)
    parts = [torch.rand(1 << 20, device=dev) for _ in range(16)]
    flat = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    for _ in range(3):
        ops.pack(parts, flat)
    torch.cuda.synchronize()
    ref = srcs[0] + srcs[1]
    ops.reduce_nway(srcs[:2], out=out, op="sum")
    torch.cuda.synchronize()
    print("pmc workload ok:", bool(torch.equal(out, ref)))


if __name__ == "__main__":
    main()
