#!/usr/bin/env python3
"""K1 tuning sweep (interleaved rounds in one process): grid size x engine for
2/4/8-source fp32 reduces of 256 MiB per source (LDS-DMA / register pipelines with
normal / non-temporal stores; the streaming kernel, grid over the whole buffer, with
normal / non-temporal stores / non-temporal loads and stores), plus torch baselines."""
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
n = (256 << 20) // 4
out = {}
for nsrc in (2, 4, 8):
    srcs = [torch.rand(n, device=dev) for _ in range(nsrc)]
    dst = torch.empty_like(srcs[0])
    res = {}
    for _ in range(4):
        for impl in ("lds", "lds_nt", "lds_ntl", "regs_nt", "regs_ntl", "stream_nt", "stream_ntl"):
            for g in ((256, 512) if not impl.startswith("stream") else (0,)):
                t = timeit(lambda: ops.reduce_nway(srcs, out=dst, impl=impl, max_blocks=g))
                res.setdefault(f"n{nsrc}_{impl}_g{g}", []).append((nsrc + 1) * n * 4 / t / 1e9)
        if nsrc == 2:
            t = timeit(lambda: torch.add(srcs[0], srcs[1], out=dst))
            res.setdefault("n2_torch_add", []).append(3 * n * 4 / t / 1e9)
        else:
            t = timeit(lambda: torch.sum(torch.stack(srcs), 0, out=dst))
            res.setdefault(f"n{nsrc}_torch_stack_sum", []).append((nsrc + 1) * n * 4 / t / 1e9)
    for k, v in res.items():
        out[k] = round(statistics.median(v), 1)
    del srcs, dst
    torch.cuda.empty_cache()
print(json.dumps(out))
