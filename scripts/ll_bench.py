#!/usr/bin/env python3
"""Small-message latency of all six collectives: LL protocol vs the staged protocols.

Ranks share ONE GPU on the 1-GPU boxes (PDCC_ALGO=ipc), so this measures the
protocols' own cost (flag round trips, staging copy, barriers), not xGMI latency.
`--modes ll,oneshot`: ll = PDCC_IPC_LL_MAX=--ll-max (default 64K), oneshot = PDCC_IPC_LL_MAX=0.
Per (mode, size): median over `--iters` of one isolated synchronous all_reduce, end to
end (host call + kernel + the ranks' arrival skew), and the per-call time of 50
back-to-back calls (median of 5), max over ranks. One JSON line per mode.

    python scripts/ll_bench.py [--world 2] [--sizes 4,1K,16K,64K] [--iters 300]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, sizes, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    out, ok = {}, True
    for nbytes in sizes:
        x = torch.full((max(1, nbytes // 4),), float(rank + 1), device=dev)
        for _ in range(20):
            dist.all_reduce(x)
        x.fill_(float(rank + 1))
        dist.all_reduce(x)
        ok = ok and bool(torch.all(x == size * (size + 1) / 2))
        algo = b.last_algo()
        lat, pipe = [], []
        for k in range(iters):  # isolated calls: launch + arrival skew + protocol
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dist.all_reduce(x)
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        for _ in range(5):  # back-to-back calls: the protocol's per-call cost once the ranks are in step
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                dist.all_reduce(x)
            torch.cuda.synchronize()
            pipe.append((time.perf_counter() - t0) / 50)
        t = torch.tensor([statistics.median(lat), statistics.median(pipe)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out[f"{nbytes}B_us"] = round(t[0].item() * 1e6, 2)
        out[f"{nbytes}B_pipelined_us"] = round(t[1].item() * 1e6, 2)
        out[f"{nbytes}B_algo"] = algo
        # all_gather of the same per-rank payload into a flat output
        src = torch.full((max(1, nbytes // 4),), float(rank), device=dev)
        flat = torch.empty(src.numel() * size, device=dev)
        for _ in range(20):
            dist.all_gather_into_tensor(flat, src)
        ok = ok and bool(torch.equal(flat.view(size, -1)[:, 0].cpu(), torch.arange(size, dtype=torch.float32)))
        ag_algo = b.last_algo()
        pipe = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                dist.all_gather_into_tensor(flat, src)
            torch.cuda.synchronize()
            pipe.append((time.perf_counter() - t0) / 50)
        t = torch.tensor([statistics.median(pipe)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out[f"ag_{nbytes}B_pipelined_us"] = round(t[0].item() * 1e6, 2)
        out[f"ag_{nbytes}B_algo"] = ag_algo
        # the rooted collectives of the reference (main.py:14,37,52,81), root 0, same per-rank payload
        n = max(1, nbytes // 4)
        y = torch.full((n,), float(rank + 1), device=dev)
        glist = [torch.empty(n, device=dev) for _ in range(size)] if rank == 0 else None
        slist = [torch.full((n,), float(r), device=dev) for r in range(size)] if rank == 0 else None
        s_out = torch.empty(n, device=dev)
        rooted = {
            "reduce": lambda: dist.reduce(y, dst=0),
            "broadcast": lambda: dist.broadcast(y, src=0),
            "gather": lambda: dist.gather(src, gather_list=glist, dst=0),
            "scatter": lambda: dist.scatter(s_out, scatter_list=slist, src=0),
        }
        for name, fn in rooted.items():
            for _ in range(20):
                fn()
            r_algo = b.last_algo()
            pipe = []
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(50):
                    fn()
                torch.cuda.synchronize()
                pipe.append((time.perf_counter() - t0) / 50)
            t = torch.tensor([statistics.median(pipe)], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            out[f"{name}_{nbytes}B_pipelined_us"] = round(t[0].item() * 1e6, 2)
            out[f"{name}_{nbytes}B_algo"] = r_algo
        ok = ok and bool(torch.all(s_out == rank))
        if rank == 0:
            ok = ok and all(bool(torch.all(g == r)) for r, g in enumerate(glist))
    out["correct"] = ok
    return out


def parse_size(s):
    s = s.strip().upper()
    mul = {"K": 1 << 10, "M": 1 << 20}.get(s[-1], 1)
    return int(s[:-1] if mul > 1 else s) * mul


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--sizes", default="4,1K,16K,64K")
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--modes", default="ll,oneshot")
    ap.add_argument("--ll-max", default="64K", help="PDCC_IPC_LL_MAX of the ll mode (<= 256K)")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    sizes = [parse_size(s) for s in a.sizes.split(",")]
    for mode in a.modes.split(","):
        env = {"PDCC_ALGO": "ipc", "PDCC_IPC_LL_MAX": a.ll_max if mode == "ll" else "0"}
        res = launch(work, a.world, args=(sizes, a.iters), bind_device=True, timeout_s=120, env=env,
                     join_timeout_s=600)
        print(json.dumps({"mode": mode, "world": a.world, **res[0]}), flush=True)


if __name__ == "__main__":
    main()
