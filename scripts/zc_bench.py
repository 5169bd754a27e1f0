#!/usr/bin/env python3
"""Zero-copy vs staged IPC collectives, several ranks sharing ONE GPU (PDCC_ALGO=ipc).

On one GPU every "peer" read is local HBM, so the time is the HBM traffic of the
protocol: the staged all-reduce copies the input into staging, reduces the own
tiles into staging and copies every reduced tile out (per rank: 3 reads + 2.5
writes of S at W = 2), the zero-copy one reads the peers' tensors in place and
writes only the own and fetched tiles (1.5 reads + 1 write of S). The same
protocol runs over xGMI on a multi-GPU node, where the saved local copy is a
serial HBM phase in front of the link-bound one.

    python scripts/zc_bench.py [--world 2] [--sizes 1M,4M,...]

Modes: staged, zc (pull protocols reading the peers' tensors in place), push (the
zero-copy push all-reduce: remote writes only). Prints one JSON line per (mode,
collective, size) and summary lines.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, sizes, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    res, enq = {}, {}
    ok = True
    for nbytes in sizes:
        n = nbytes // 4
        x = torch.full((n,), float(rank + 1), device=dev)
        ag_in = torch.full((n // size,), float(rank), device=dev)
        ag_out = torch.empty(n // size * size, device=dev)
        rs_in = torch.ones(n // size * size, device=dev)
        rs_out = torch.empty(n // size, device=dev)
        a2a_out = torch.empty_like(rs_in)
        sc_list = list(rs_in.chunk(size)) if rank == 0 else None  # flat views: read in place
        cases = {
            "all_reduce": lambda: dist.all_reduce(x),
            "reduce": lambda: dist.reduce(x, dst=0),
            "scatter": lambda: dist.scatter(rs_out, scatter_list=sc_list, src=0),
            "broadcast": lambda: dist.broadcast(x, 0),
            "all_gather": lambda: dist.all_gather_into_tensor(ag_out, ag_in),
            "reduce_scatter": lambda: dist.reduce_scatter_tensor(rs_out, rs_in),
            "all_to_all": lambda: dist.all_to_all_single(a2a_out, rs_in),
        }
        for name, fn in cases.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            k = iters if nbytes <= (16 << 20) else max(3, iters // 4)
            host = []
            t0 = time.perf_counter()
            for _ in range(k):
                h0 = time.perf_counter()
                fn()
                host.append(time.perf_counter() - h0)
            torch.cuda.synchronize()
            res[f"{name}/{nbytes}"] = (time.perf_counter() - t0) / k * 1e6
            enq[f"{name}/{nbytes}"] = sorted(host)[len(host) // 2] * 1e6  # host enqueue (median)
        # correctness after the timed loops (inputs re-made: the loops accumulate)
        x.fill_(float(rank + 1))
        dist.all_reduce(x)
        ok = ok and bool(torch.all(x == size * (size + 1) / 2).item())
        dist.all_gather_into_tensor(ag_out, ag_in)
        ok = ok and bool(torch.equal(ag_out.view(size, -1)[:, 0].cpu(), torch.arange(size, dtype=torch.float32)))
        dist.reduce_scatter_tensor(rs_out, rs_in)
        ok = ok and bool(torch.all(rs_out == size).item())
    st = be.stats()
    # host enqueue per call (validation, engine choice, zero-copy handle exchange, launch), median
    host_us = {k: round(v, 1) for k, v in enq.items() if k.startswith("all_reduce/")}
    return {"us": res, "correct": ok, "zc_calls": sum(v[0] for k, v in st.items() if k.endswith("_zc")),
            "host_us_per_call": host_us, "describe": be.describe()[-160:]}


def parse_sizes(s):
    out = []
    for tok in s.split(","):
        mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(tok[-1].upper(), 1)
        out.append(int(float(tok[:-1] if mult > 1 else tok) * mult))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--sizes", default="1M,4M,16M,64M,256M")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="staged,zc,push", help="comma list of staged|zc|push (one mode per rocprof run)")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    sizes = parse_sizes(a.sizes)
    runs = {}
    for mode in a.modes.split(","):
        # push: the zero-copy push all-reduce (remote writes only); other collectives as in zc
        env = {"PDCC_ALGO": "ipc_push" if mode == "push" else "ipc", "PDCC_IPC_ZC": "0" if mode == "staged" else "1",
               "PDCC_IPC_1SHOT_MAX": "256K"}
        out = launch(work, a.world, args=(sizes, a.iters), bind_device=True, timeout_s=60, env=env,
                     join_timeout_s=500)
        runs[mode] = out[0]
        for key, us in out[0]["us"].items():
            coll, nb = key.split("/")
            print(json.dumps({"world_on_one_gpu": a.world, "mode": mode, "coll": coll, "bytes": int(nb),
                              "us": round(us, 1)}), flush=True)
        print(json.dumps({"mode": mode, "correct": out[0]["correct"], "zc_calls": out[0]["zc_calls"],
                          "host_us_per_call": out[0]["host_us_per_call"]}), flush=True)
    if "staged" in runs and "zc" in runs:
        speed = {k: round(runs["staged"]["us"][k] / runs["zc"]["us"][k], 2) for k in runs["zc"]["us"]}
        print(json.dumps({"world_on_one_gpu": a.world, "speedup_staged_over_zc": speed,
                          "correct": runs["staged"]["correct"] and runs["zc"]["correct"]}), flush=True)
    if "zc" in runs and "push" in runs:
        speed = {k: round(runs["zc"]["us"][k] / runs["push"]["us"][k], 2) for k in runs["push"]["us"]
                 if k.startswith("all_reduce/")}
        print(json.dumps({"world_on_one_gpu": a.world, "all_reduce_speedup_pull_over_push": speed,
                          "correct": runs["push"]["correct"]}), flush=True)
