#!/usr/bin/env python3
"""Static vs dynamic zero-copy 2-shot all_reduce, ranks sharing one GPU.

PDCC_ALGO=ipc runs the static protocol (a fixed tile range per workgroup, block-pairwise
barrier between the phases); PDCC_ALGO=ipc_dyn the dynamic one (work items claimed per
workgroup from a counter, per-chunk ready words; kern::kDynOffset). Median wall time of
`--iters` synchronous all_reduces (max over ranks) per size, correctness checked, and the
busbw-style HBM rate of the whole call (both ranks' traffic on the one GPU).

    python scripts/dyn_bench.py [--world 2] [--mib 16,64,256] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work_other(rank, size, mibs, iters, coll):
    """all_gather (S / W per rank in, S out) or reduce_scatter (S in, S / W out): median us."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    out = {}
    for mib in mibs:
        n = (mib << 20) // 4
        big, part = torch.empty(n, device=dev), torch.empty(n // size, device=dev)
        part.fill_(float(rank + 1))
        big.fill_(float(rank + 1))

        def call():
            if coll == "all_gather":
                dist.all_gather_into_tensor(big, part)
            else:
                dist.reduce_scatter_tensor(part, big)

        for _ in range(3):
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
        if coll == "all_gather":
            ok = bool(torch.equal(big.view(size, -1)[:, 0].cpu(), torch.arange(1, size + 1, dtype=torch.float32)))
        else:
            part.fill_(0.0)
            big.fill_(float(rank + 1))
            call()
            ok = bool(torch.all(part == float(size * (size + 1) // 2)).item())
        out[mib] = {"us": round(statistics.median(lat) * 1e6, 1), "engine": engine, "correct": ok}
        del big, part
        torch.cuda.empty_cache()
    return out


def work(rank, size, mibs, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    out = {}
    for mib in mibs:
        n = (mib << 20) // 4
        x = torch.empty(n, device=dev)
        for _ in range(3):
            x.fill_(float(rank + 1))
            dist.all_reduce(x)
        torch.cuda.synchronize()
        lat, ok = [], True
        for i in range(iters):
            x.fill_(float(rank + 1 + i % 5))
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            dist.all_reduce(x)
            torch.cuda.synchronize()
            engine = b.last_algo()
            t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            lat.append(t.item())
            ok = ok and bool(torch.all(x == float(sum(r + 1 + i % 5 for r in range(size)))))
        us = statistics.median(lat) * 1e6
        out[mib] = {"us": round(us, 1), "engine": engine, "correct": ok}
        del x
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mib", default="16,64,256")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--coll", default="all_reduce", help="all_reduce | all_gather | reduce_scatter")
    ap.add_argument("--algos", default="ipc,ipc_dyn",
                    help="PDCC_ALGO values; ipc_dyn@N also sets PDCC_IPC_DYN=N (chunks per workgroup); "
                         "';KEY=VAL' suffixes set more environment (ipc_dyn;PDCC_IPC_DYN_MIN_ROWS=32)")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    mibs = [int(m) for m in a.mib.split(",")]
    res = {}
    for algo in a.algos.split(","):
        spec, *extra = algo.split(";")  # ;KEY=VAL: more environment for this engine's run
        name = spec
        env = {"PDCC_ALGO": name.split("@")[0], "PDCC_AUTOTUNE": "0"}
        env.update(kv.split("=", 1) for kv in extra)
        if "@" in name:
            env["PDCC_IPC_DYN"] = name.split("@")[1]
        if a.coll == "all_reduce":
            r = launch(work, a.world, args=(mibs, a.iters), bind_device=True, timeout_s=120, env=env,
                       join_timeout_s=500)
        else:
            r = launch(work_other, a.world, args=(mibs, a.iters, a.coll), bind_device=True, timeout_s=120, env=env,
                       join_timeout_s=500)
        res[algo] = r[0]
        for mib, v in r[0].items():
            W, S = a.world, mib << 20
            rec = {"world_on_one_gpu": W, "coll": a.coll, "algo": algo, "mib": mib, **v}
            if a.coll == "all_reduce":
                # HBM bytes of one zero-copy 2-shot call, all ranks on one GPU (scripts/ipc_phase_trace.py)
                rec["hbm_TBps"] = round((W * S * (1 + (W - 1) / W) + W * S) / (v["us"] * 1e-6) / 1e12, 2)
            print(json.dumps(rec), flush=True)
    algos = a.algos.split(",")
    if len(algos) == 2:
        sp = {m: round(res[algos[0]][m]["us"] / res[algos[1]][m]["us"], 3) for m in mibs}
        print(json.dumps({"world_on_one_gpu": a.world, "coll": a.coll, f"speedup_{algos[1]}_over_{algos[0]}": sp}),
              flush=True)


if __name__ == "__main__":
    main()
