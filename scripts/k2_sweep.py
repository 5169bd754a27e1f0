#!/usr/bin/env python3
"""K2 multi_copy tuning sweep (interleaved rounds in one process): grid cap x
LDS-DMA ring depth for several list shapes, plus the default policy
(max_blocks=0) and a torch copy of the same bytes as the HBM reference.
Bandwidth = 2 x bytes / time (read + write)."""
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
shapes = [(64, 4 << 20), (8, 32 << 20), (8, 1 << 20), (4, 256 << 20), (32, 64 << 10), (8, 128 << 20)]
for count, nbytes in shapes:
    n = nbytes // 4
    tag = f"{count}x{nbytes >> 10}K"
    srcs = [torch.rand(n, device=dev) for _ in range(count)]
    dsts = [torch.empty_like(s) for s in srcs]
    flat_src = torch.cat(srcs)
    flat_dst = torch.empty_like(flat_src)
    byts = 2 * count * nbytes
    res = {}
    for _ in range(3):
        for depth in (4, 8):
            for g in (256, 512, 1024, 2048):
                t = timeit(lambda: ops.multi_copy(srcs, dsts, max_blocks=g, depth=depth, ntl=False))
                res.setdefault(f"{tag}_d{depth}_g{g}", []).append(byts / t / 1e9)
        t = timeit(lambda: ops.multi_copy(srcs, dsts, ntl=False))
        res.setdefault(f"{tag}_default_grid", []).append(byts / t / 1e9)
        t = timeit(lambda: ops.multi_copy(srcs, dsts, ntl=True))
        res.setdefault(f"{tag}_default_grid_ntl", []).append(byts / t / 1e9)
        t = timeit(lambda: ops.multi_copy(srcs, dsts))
        res.setdefault(f"{tag}_default", []).append(byts / t / 1e9)
        t = timeit(lambda: flat_dst.copy_(flat_src))
        res.setdefault(f"{tag}_torch_flat_copy", []).append(byts / t / 1e9)
    ok = all(torch.equal(a, b) for a, b in zip(srcs, dsts))
    for k, v in res.items():
        out[k] = round(statistics.median(v), 1)
    best = max((k for k in res if "_d" in k), key=lambda k: out[k])
    out[f"{tag}_best"] = best
    out[f"{tag}_default_vs_best"] = round(out[f"{tag}_default"] / out[best], 3)
    out[f"{tag}_correct"] = ok
    del srcs, dsts, flat_src, flat_dst
    torch.cuda.empty_cache()
print(json.dumps(out))
