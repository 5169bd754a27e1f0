#!/usr/bin/env python3
"""Microbenchmark of the gfx950 kernels on one GPU (interleaved A/B rounds in
one process, cdna_hip_programming.md §5.4 rule 24).

K1 reduce_nway: LDS-DMA engine vs register-staged variant (normal stores), the LDS-DMA
engine with non-temporal stores and the streaming kernel (non-temporal stores / loads and
stores), nsrc in {2,4,8},
fp32/bf16, 256 MiB per source (past the 256 MiB Infinity Cache for nsrc>=2).
Effective bandwidth = (nsrc + 1) * bytes / time (every source read once, one write).
K2 multi_copy: 64 tensors of 4 MiB, bandwidth = 2 * bytes / time.
Prints one JSON object.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_collective_communication_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    dev = torch.device("cuda", 0)
    out = {"device": torch.cuda.get_device_name(0)}
    per_src = int(os.environ.get("KB_BYTES", str(256 << 20)))
    for dt in (torch.float32, torch.bfloat16):
        n = per_src // torch.tensor([], dtype=dt).element_size()
        for nsrc in (2, 4, 8):
            srcs = [torch.rand(n, device=dev).to(dt) for _ in range(nsrc)]
            dst = torch.empty_like(srcs[0])
            res = {k: [] for k in ("lds", "regs", "lds_nt", "stream_nt", "stream_ntl")}
            for _ in range(5):
                for impl in res:
                    t = timeit(lambda: ops.reduce_nway(srcs, out=dst, impl=impl))
                    res[impl].append((nsrc + 1) * per_src / t / 1e9)
            for impl in res:
                out[f"k1_{str(dt).split('.')[-1]}_n{nsrc}_{impl}_GBps"] = round(statistics.median(res[impl]), 1)
            del srcs, dst
            torch.cuda.empty_cache()
    srcs = [torch.rand(1 << 20, device=dev) for _ in range(64)]
    dsts = [torch.empty_like(s) for s in srcs]
    t = timeit(lambda: ops.multi_copy(srcs, dsts), 20)
    out["k2_64x4MiB_GBps"] = round(2 * 64 * (4 << 20) / t / 1e9, 1)
    t = timeit(lambda: [d.copy_(s) for s, d in zip(srcs, dsts)], 20)
    out["torch_copy_64x4MiB_GBps"] = round(2 * 64 * (4 << 20) / t / 1e9, 1)
    big = torch.rand(256 << 20, device=dev)
    big2 = torch.empty_like(big)
    t = timeit(lambda: big2.copy_(big), 10)
    out["torch_copy_1GiB_GBps"] = round(2 * big.numel() * 4 / t / 1e9, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
