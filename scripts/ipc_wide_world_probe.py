#!/usr/bin/env python3
"""Which IPC kernel goes wrong at a given world size? (ranks sharing one GPU, self-test off)

Runs each staged IPC protocol a few times at world sizes --worlds and reports, per
(world, collective), whether every rank got the exact result, plus the first bad
index / value on a failing rank. One JSON line per world.

    python scripts/ipc_wide_world_probe.py [--worlds 4,6,8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, reps):
    import torch
    import torch.distributed as dist

    d = torch.device("cuda", torch.cuda.current_device())
    res = {}

    def note(key, got, want):
        good = bool(torch.equal(got, want))
        if not good:
            bad = (got != want).nonzero().flatten()
            res.setdefault(key, []).append({"rank": rank, "nbad": int(bad.numel()), "first": int(bad[0]),
                                            "got": float(got.flatten()[bad[0]]), "want": float(want.flatten()[bad[0]])})
        return good

    tri = size * (size + 1) / 2
    for k in range(reps):
        for key, n in (("ar_1shot_1000", 1000), ("ar_2shot", 3 * size * 1024 + 257), ("ar_2shot_big", 1 << 20)):
            base = torch.arange(n, device=d).remainder(7).float()
            x = base + (rank + 1 + k)
            dist.all_reduce(x)
            note(key, x, base * size + tri + size * k)
        m = 780
        out = torch.full((m * size,), -1.0, device=d)
        dist.all_gather_into_tensor(out, torch.full((m,), float(rank + k), device=d))
        note("allgather_780", out, (torch.arange(size, device=d).float() + k).repeat_interleave(m))
        y = torch.full((5000,), float(rank + k), device=d) if rank == 0 else torch.zeros(5000, device=d)
        dist.broadcast(y, src=0)
        note("broadcast_5000", y, torch.full((5000,), float(k), device=d))
        # ragged bulk sizes (partial rows / tiles) through the rooted and chunked collectives
        nb = (1 << 20) + 3 * 1024 + 5
        root = (k * 3 + 1) % size
        base = torch.arange(nb, device=d).remainder(7).float()
        z = base + (rank + 1 + k)
        dist.reduce(z, dst=root)
        note("reduce_big", z, base * size + tri + size * k if rank == root else base + (rank + 1 + k))
        z = base + k if rank == root else torch.zeros(nb, device=d)
        dist.broadcast(z, src=root)
        note("broadcast_big", z, base + k)
        mb = (1 << 18) + 1031
        ins = [torch.full((mb,), float(100 * rank + q + k), device=d) for q in range(size)]
        o = torch.empty(mb, device=d)
        dist.reduce_scatter(o, ins)
        note("reduce_scatter_big", o, torch.full((mb,), float(100 * tri - 100 * size + size * (rank + k)), device=d))
        outs = [torch.empty(mb, device=d) for _ in range(size)]
        dist.all_to_all(outs, ins)
        note("all_to_all_big", torch.stack(outs),
             torch.stack([torch.full((mb,), float(100 * q + rank + k), device=d) for q in range(size)]))
        g = [torch.empty(mb, device=d) for _ in range(size)] if rank == root else None
        dist.gather(ins[0], gather_list=g, dst=root)
        if rank == root:
            note("gather_big", torch.stack(g), torch.stack([torch.full((mb,), float(100 * q + k), device=d)
                                                            for q in range(size)]))
        s_in = [torch.full((mb,), float(10 * q + k), device=d) for q in range(size)] if rank == root else None
        dist.scatter(o, scatter_list=s_in, src=root)
        note("scatter_big", o, torch.full((mb,), float(10 * rank + k), device=d))
    torch.cuda.synchronize()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="4,6,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--env", default="", help="extra K=V,K=V for the ranks")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    for w in [int(x) for x in a.worlds.split(",")]:
        env = {"PDCC_ALGO": "ipc", "PDCC_IPC_SELFTEST": "0", "PDCC_IPC_LL_MAX": "0", "PDCC_IPC_ZC": "0",
               "PDCC_IPC_SPIN_MS": "5000"}
        for kv in filter(None, a.env.split(",")):
            k, v = kv.split("=", 1)
            env[k] = v
        res = launch(work, w, args=(a.reps,), bind_device=True, timeout_s=120, env=env, join_timeout_s=300)
        merged = {}
        for r in res:
            for key, v in r.items():
                merged.setdefault(key, []).extend(v)
        print(json.dumps({"world": w, "env": a.env, "failures": merged}), flush=True)


if __name__ == "__main__":
    main()
