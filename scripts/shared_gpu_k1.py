#!/usr/bin/env python3
"""What ranks sharing ONE GPU cost a streaming kernel: K1 (2-source LDS-DMA reduce, the
all-reduce's phase 1) run by W processes at once, each on its own buffers with 256 / W
workgroups (the grid the IPC kernels get on a shared GPU), against one process running the
same total bytes with 256 workgroups. Start is aligned with a barrier; each process times
`--iters` back-to-back launches; the aggregate rate = all processes' bytes / the slowest
process's time. If W concurrent processes reach clearly less than one, the IPC protocols'
shortfall from K1 on one shared GPU is (partly) a multi-process artifact that distinct GPUs
do not have.

    python scripts/shared_gpu_k1.py [--world 2] [--mib 256] [--iters 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, mib, iters, blocks):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd import ops

    dev = torch.device("cuda", torch.cuda.current_device())
    n = (mib << 20) // 4 // size  # each process: its share of the total
    s = [torch.rand(n, device=dev) for _ in range(2)]
    o = torch.empty(n, device=dev)
    for _ in range(3):
        ops.reduce_nway(s, out=o, impl="lds_ntl", max_blocks=blocks)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        ops.reduce_nway(s, out=o, impl="lds_ntl", max_blocks=blocks)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"rank": rank, "s": dt, "s_max": t.item(), "bytes_per_iter": 3 * n * 4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    for w in (1, a.world):
        res = launch(work, w, args=(a.mib, a.iters, 256 // w), bind_device=True, timeout_s=120, join_timeout_s=300)
        tot = sum(r["bytes_per_iter"] for r in res) * a.iters
        print(json.dumps({"processes": w, "workgroups_each": 256 // w, "total_mib_per_source": a.mib,
                          "aggregate_TBps": round(tot / res[0]["s_max"] / 1e12, 2),
                          "per_process_s": [round(r["s"], 4) for r in res]}), flush=True)


if __name__ == "__main__":
    main()
