#!/usr/bin/env python3
"""PDCC_IPC_ASYNC_GRID evidence (verdict r3 Next #4): the same 4 MiB IPC all_reduce issued
synchronously and with async_op=True, two ranks sharing one GPU. Under
`rocprofv3 --kernel-trace` the async launches carry the capped grid (Grid_Size = cap x 256
threads) and the synchronous ones the full grid; describe() counts the capped launches.

    PDCC_IPC_ASYNC_GRID=32 rocprofv3 --kernel-trace --output-format csv -d <dir> -- \\
        python3 scripts/async_grid_probe.py
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, calls):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    x = torch.full(((4 << 20) // 4,), float(rank + 1), device=d)
    ok = True
    for i in range(calls):
        x.fill_(float(rank + 1))
        dist.all_reduce(x)  # caller's stream: full grid
        ok = ok and bool(torch.all(x == size * (size + 1) / 2))
        x.fill_(float(rank + 1))
        dist.all_reduce(x, async_op=True).wait()  # comm stream: capped grid
        ok = ok and bool(torch.all(x == size * (size + 1) / 2))
    torch.cuda.synchronize()
    m = re.search(r"async_capped=(\d+)", b.describe())
    return {"ok": ok, "async_capped": int(m.group(1)) if m else -1, "engine": b.last_algo(),
            "async_grid": os.environ.get("PDCC_IPC_ASYNC_GRID", "0")}


def main():
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    res = launch(work, 2, args=(8,), bind_device=True, timeout_s=60, env={"PDCC_ALGO": "ipc"}, join_timeout_s=300)
    print(json.dumps(res[0]), flush=True)


if __name__ == "__main__":
    main()
