#!/usr/bin/env python3
"""The autotuner's verdict for the copy collectives above 4 MiB without RCCL, against the engines
forced one by one (round 5: the 1 GiB broadcast of the W = 4 / 8 shared-GPU rehearsals came out
staged and 2.2x slower than round 4's zero-copy run).

For each collective (broadcast, all_gather_into_tensor, reduce, reduce_scatter_tensor) at the given
size: one group with the autotuner on -- its first call races the candidates; then the median of
`iters` timed calls and the table row -- and one group per forced engine (ipc, ipc_staged, ipc_dyn
where it applies) timed the same way. W ranks share one GPU (GPU_MAX_HW_QUEUES=1 per rank).

    python scripts/race_probe.py --world 4 --mib 1024 [--iters 5]
"""
import argparse
import datetime
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COLLS = ("broadcast", "all_gather", "reduce", "reduce_scatter")


def work(rank, size, mib, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    n = (mib << 20) // 4
    x = torch.rand(n, device=dev)
    per = n // size
    ag_out = torch.empty(per * size, device=dev)
    rs_out = torch.empty(per, device=dev)

    def call(coll, g):
        if coll == "broadcast":
            dist.broadcast(x, src=0, group=g)
        elif coll == "all_gather":
            dist.all_gather_into_tensor(ag_out, x[:per], group=g)
        elif coll == "reduce":
            dist.reduce(x, dst=0, group=g)
        else:
            dist.reduce_scatter_tensor(rs_out, x[: per * size], group=g)

    out = {}
    for engine in ("auto", "ipc", "ipc_staged", "ipc_dyn"):
        g = dist.new_group(list(range(size)), timeout=datetime.timedelta(seconds=120))
        gb = be.native_backend(g, "cuda")
        gb.set_algo(engine)
        for coll in COLLS:
            if engine == "ipc_dyn" and coll not in ("all_gather", "reduce_scatter"):
                continue
            call(coll, g)  # (auto: the race)
            torch.cuda.synchronize()
            lat = []
            for _ in range(iters):
                x.uniform_(0.0, 1e-3)
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                call(coll, g)
                torch.cuda.synchronize()
                t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
                eng = gb.last_algo()
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                lat.append(t.item())
            out[f"{coll}/{engine}"] = {"us": round(statistics.median(lat) * 1e6, 1), "engine": eng}
        if engine == "auto":
            out["table"] = gb.autotune_table()
        dist.destroy_process_group(g)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    env = {"GPU_MAX_HW_QUEUES": "1", "PDCC_LOG_LEVEL": "1"}
    res = launch(work, a.world, args=(a.mib, a.iters), bind_device=True, timeout_s=120, env=env, join_timeout_s=500)
    print(json.dumps({"world_on_one_gpu": a.world, "mib": a.mib, **res[0]}), flush=True)


if __name__ == "__main__":
    main()
