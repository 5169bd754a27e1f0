#!/usr/bin/env python3
"""Drive the hipIpc peer-memory collectives with several ranks on ONE GPU
(PDCC_ALGO=ipc) -- used for rocprofv3 kernel traces of the IPC kernels and as
a latency probe of their protocol overhead (on one GPU the "peer" reads are
local HBM, so this is NOT an xGMI bandwidth number).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, sizes):
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device())
    res = {}
    for nbytes in sizes:
        x = torch.ones(nbytes // 4, device=dev)
        for name, fn in (
            ("all_reduce", lambda: dist.all_reduce(x)),
            ("broadcast", lambda: dist.broadcast(x, 0)),
            ("all_gather", lambda: dist.all_gather_into_tensor(ag, x)),
            ("reduce_scatter", lambda: dist.reduce_scatter_tensor(rs, rsin)),
        ):
            ag = torch.empty(size * x.numel(), device=dev)
            rs = torch.empty(max(1, x.numel() // size), device=dev)
            rsin = torch.ones(rs.numel() * size, device=dev)
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            iters = 20 if nbytes <= (1 << 20) else 5
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            res[f"{name}_{nbytes}B_us"] = round((time.perf_counter() - t0) / iters * 1e6, 1)
    x = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    res["correct"] = bool(torch.all(x == size * (size + 1) / 2).item())
    return res


if __name__ == "__main__":
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    world = int(os.environ.get("IPC_DEMO_WORLD", "2"))
    sizes = [4096, 256 << 10, 4 << 20, 64 << 20]
    out = launch(work, world, args=(sizes,), bind_device=True, timeout_s=60,
                 env={"PDCC_ALGO": "ipc"}, join_timeout_s=500)
    print(json.dumps({"world_on_one_gpu": world, "rank0": out[0]}))
