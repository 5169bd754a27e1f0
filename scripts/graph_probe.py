#!/usr/bin/env python3
"""Where does the time go around a hipGraph capture of IPC collectives?
2 ranks sharing cuda:0 (IPC engine). For 4 KiB all_reduces: host issue time per
call (no sync) and synchronized per-call time, before any capture, after a
capture, and for replays. Prints one JSON line per rank."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, n_ops=16, iters=40):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel.graphs import capture

    dev = torch.device("cuda", torch.cuda.current_device())
    bufs = [torch.zeros(1024, device=dev) for _ in range(n_ops)]

    def step():
        for b in bufs:
            dist.all_reduce(b)

    def measure(tag, fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        issue = 0.0
        t0 = time.perf_counter()
        for _ in range(iters):
            a = time.perf_counter()
            fn()
            issue += time.perf_counter() - a
        torch.cuda.synchronize()
        total = time.perf_counter() - t0
        return {f"{tag}_issue_us_per_op": round(issue / iters / n_ops * 1e6, 2),
                f"{tag}_total_us_per_op": round(total / iters / n_ops * 1e6, 2)}

    out = {}
    out.update(measure("eager", step))
    g = capture(step, warmup=2)
    out.update(measure("replay", g.replay))
    out.update(measure("eager_after", step))
    return out


if __name__ == "__main__":
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    res = launch(work, 2, bind_device=True, timeout_s=60, env={"PDCC_ALGO": "ipc"}, join_timeout_s=300)
    for r, x in enumerate(res):
        print(json.dumps({"rank": r, **x}))
