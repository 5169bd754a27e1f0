#!/usr/bin/env python3
"""K2 multi_copy tuning sweep (interleaved rounds in one process): grid cap x
LDS-DMA ring depth for 64 x 4 MiB and 8 x 32 MiB lists, plus a 1 GiB torch
copy as the HBM reference. Bandwidth = 2 x bytes / time."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_collective_communication_amd import ops  # noqa: E402


def timeit(fn, iters=8):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


dev = torch.device("cuda", 0)
out = {}
for count, mib in ((64, 4), (8, 32)):
    n = (mib << 20) // 4
    srcs = [torch.rand(n, device=dev) for _ in range(count)]
    dsts = [torch.empty_like(s) for s in srcs]
    byts = 2 * count * n * 4
    res = {}
    for _ in range(4):
        for depth in (4, 8):
            for g in (256, 512, 1024, 2048):
                t = timeit(lambda: ops.multi_copy(srcs, dsts, max_blocks=g, depth=depth))
                res.setdefault(f"{count}x{mib}M_d{depth}_g{g}", []).append(byts / t / 1e9)
    ok = all(torch.equal(a, b) for a, b in zip(srcs, dsts))
    for k, v in res.items():
        out[k] = round(statistics.median(v), 1)
    out[f"{count}x{mib}M_correct"] = ok
    del srcs, dsts
big = torch.rand(1 << 28, device=dev)
bd = torch.empty_like(big)
out["torch_copy_1GiB"] = round(statistics.median([2 * big.numel() * 4 / timeit(lambda: bd.copy_(big)) / 1e9
                                                  for _ in range(4)]), 1)
print(json.dumps(out))
