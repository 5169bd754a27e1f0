#!/usr/bin/env python3
"""Coalesced collectives vs a per-member loop (verdict r3 Next #5), ranks sharing one GPU.

64 members of 16 KiB (fp32) per call, the DDP / ZeRO bucket shape: torch's
_coalescing_manager fast path (all_reduce, all_gather_into_tensor, reduce_scatter_tensor)
packs them into ONE collective (csrc/backend/coalesced.cpp), against issuing one collective per
member. Median wall time of 20 calls each (max over ranks), plus the number of collectives the
backend recorded per call. Under `rocprofv3 --kernel-trace --stats` the coalesced phase shows
one collective kernel per call (plus the K2 pack / unpack launches).

    python scripts/coalesced_bench.py [--world 2] [--n 64] [--kib 16] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, n, kib, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    m = (kib << 10) // 4
    xs = [torch.rand(m, device=d) for _ in range(n)]
    outs = [torch.empty(m * size, device=d) for _ in range(n)]
    ins_rs = [torch.rand(m * size, device=d) for _ in range(n)]
    outs_rs = [torch.empty(m, device=d) for _ in range(n)]
    pg = dist.distributed_c10d._get_default_group()
    cases = {
        "all_reduce": (lambda: [dist.all_reduce(x) for x in xs],
                       lambda: _coal(d, lambda: [dist.all_reduce(x) for x in xs]),
                       lambda: dist.all_reduce_coalesced(xs)),
        "all_gather": (lambda: [dist.all_gather_into_tensor(o, x) for o, x in zip(outs, xs)],
                       lambda: _coal(d, lambda: [dist.all_gather_into_tensor(o, x) for o, x in zip(outs, xs)]),
                       lambda: pg.allgather_into_tensor_coalesced(outs, xs).wait()),
        "reduce_scatter": (lambda: [dist.reduce_scatter_tensor(o, x) for o, x in zip(outs_rs, ins_rs)],
                           lambda: _coal(d, lambda: [dist.reduce_scatter_tensor(o, x)
                                                     for o, x in zip(outs_rs, ins_rs)]),
                           lambda: pg.reduce_scatter_tensor_coalesced(outs_rs, ins_rs,
                                                                      dist.ReduceScatterOptions()).wait()),
    }
    res = {}
    # modes: a Python loop of single collectives; torch's _coalescing_manager (records every op in
    # Python, then ONE backend call); the backend's coalesced entry point called once from Python
    for name, (loop, coal, direct) in cases.items():
        for mode, fn in (("loop", loop), ("coalesced", coal), ("direct", direct)):
            fn()
            torch.cuda.synchronize()
            before = _colls(b)
            lat = []
            for _ in range(iters):
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                engine = b.last_algo()  # (before the host-transport MAX below records "shm")
                t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                lat.append(t.item())
            res[f"{name}_{mode}_us"] = round(statistics.median(lat) * 1e6, 1)
            res[f"{name}_{mode}_collectives_per_call"] = round((_colls(b) - before) / iters, 2)
            res[f"{name}_{mode}_engine"] = engine
        res[f"{name}_speedup"] = round(res[f"{name}_loop_us"] / res[f"{name}_coalesced_us"], 2)
        res[f"{name}_speedup_direct"] = round(res[f"{name}_loop_us"] / res[f"{name}_direct_us"], 2)
    res["autotune"] = [{k: e[k] for k in ("coll", "lo", "algo", "ref_us", "ipc_us", "staged_us")}
                       for e in b.autotune_table()]
    return res


def _colls(b):
    """GPU collectives recorded so far (not the timing barrier / host-transport MAX)."""
    return sum(v[0] for k, v in b.stats().items()
               if not k.startswith(("coalesced/", "rccl_comm/", "barrier")) and not k.endswith("/shm"))


def _coal(d, body):
    import torch.distributed as dist

    with dist._coalescing_manager(device=d, async_ops=False):
        body()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--kib", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    res = launch(work, a.world, args=(a.n, a.kib, a.iters), bind_device=True, timeout_s=120, join_timeout_s=400)
    out = dict(res[0])
    out.update(world_on_one_gpu=a.world, members=a.n, member_bytes=a.kib << 10)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
