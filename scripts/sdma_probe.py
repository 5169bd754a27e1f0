#!/usr/bin/env python3
"""Copy engines vs CU kernels for the copy collectives, ranks sharing one GPU (or one per GPU).

For each engine in ``--algos`` (PDCC_ALGO values: ``ipc`` = the zero-copy IPC kernels,
``ipc_sdma`` = hipMemcpyAsync pulls between IPC-mapped user buffers, gpu_ops.cpp sdma_run)
and each collective -- broadcast, all_gather (flat), all_to_all -- at ``--mib`` per rank:
median wall time of ``--iters`` synchronous calls (max over ranks), the engine that served
them (``last_algo()``) and a bitwise check. Run it under
``rocprofv3 --memory-copy-trace --kernel-trace`` to see which engine HIP used for the pulls
(copy-engine operations appear in the memory-copy trace; blit kernels in the kernel trace).

    python scripts/sdma_probe.py [--world 2] [--mib 4,64] [--iters 10] [--algos ipc,ipc_sdma]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, mibs, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    out = {}
    for mib in mibs:
        n = (mib << 20) // 4
        src = torch.arange(n, device=dev, dtype=torch.float32) + rank * n
        full = torch.empty(n * size, device=dev)
        a2a_in = torch.arange(n * size, device=dev, dtype=torch.float32) + rank * n * size
        bc = torch.empty(n, device=dev)
        calls = {
            "broadcast": lambda: dist.broadcast(bc, src=0),
            "all_gather": lambda: dist.all_gather_into_tensor(full, src),
            "all_to_all": lambda: dist.all_to_all_single(full, a2a_in),
        }
        for name, call in calls.items():
            if name == "broadcast":
                bc.copy_(src if rank == 0 else torch.zeros_like(src))
            for _ in range(2):
                call()
            torch.cuda.synchronize()
            lat = []
            for _ in range(iters):
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                call()
                torch.cuda.synchronize()
                engine = b.last_algo()
                t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                lat.append(t.item())
            base = torch.arange(n, device=dev, dtype=torch.float32)
            if name == "broadcast":
                ok = bool(torch.equal(bc, base))
            elif name == "all_gather":
                ok = all(bool(torch.equal(full[r * n:(r + 1) * n], base + r * n)) for r in range(size))
            else:
                ok = all(bool(torch.equal(full[q * n:(q + 1) * n], base + q * n * size + rank * n)) for q in range(size))
            us = statistics.median(lat) * 1e6
            moved = mib if name == "broadcast" else mib * (size - 1)  # MiB one receiving rank pulls
            out[f"{name}/{mib}MiB"] = {"us": round(us, 1), "engine": engine, "correct": ok,
                                       "GBps_per_rank_in": round(moved * (1 << 20) / (us * 1e-6) / 1e9, 1)}
        del src, full, a2a_in, bc
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mib", default="4,64")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--algos", default="ipc,ipc_sdma")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    mibs = [int(m) for m in a.mib.split(",")]
    res = {}
    for algo in a.algos.split(","):
        env = {"PDCC_ALGO": algo, "PDCC_AUTOTUNE": "0"}
        r = launch(work, a.world, args=(mibs, a.iters), bind_device=True, timeout_s=120, env=env, join_timeout_s=300)
        res[algo] = r[0]
        print(json.dumps({"algo": algo, "world": a.world, **r[0]}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"world": a.world, "mib": mibs, "iters": a.iters, "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
