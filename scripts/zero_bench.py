#!/usr/bin/env python3
"""Data-parallel training step: ZeRO-style ShardedOptimizer vs replicated DP.

A stack of bf16 Linear layers (default 24 x 4096^2 = 403 M parameters, 806 MB
of bf16 weights), one rank per GPU (or several ranks sharing one GPU on the
1-GPU boxes), AdamW. Modes:

* ``zero``         -- parallel.zero.ShardedOptimizer, bucket reduce-scatters
                      launched during backward (overlap), per-bucket all-gather
* ``zero_nooverlap`` -- same, every reduce-scatter issued in step()
* ``ddp``          -- parallel.ddp.GradBucketer (overlapped bucketed all-reduce,
                      AVG) + a replicated fp32-state AdamW on every rank

Per mode: median step time (forward + backward + optimizer + collectives,
bracketed by cuda.synchronize), the optimizer/collective tail after backward,
and the optimizer-state bytes each rank holds. One JSON line per mode.

    python scripts/zero_bench.py [--world 2] [--layers 24] [--dim 4096] [--steps 8]
        [--async-grids 0,64,32] [--repeat 2]

``--async-grids``: one run per PDCC_IPC_ASYNC_GRID value (workgroup cap of the IPC launches
of async collectives -- the overlapped buckets; 0 = uncapped). Each line also reports
which engines served the collectives (per-engine call counts of the default group).
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, mode, layers, dim, steps, batch):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import ddp
    from pytorch_distributed_collective_communication_amd.parallel.zero import ShardedOptimizer

    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(0)
    model = torch.nn.Sequential(*[torch.nn.Linear(dim, dim, bias=False) for _ in range(layers)]).to(dev, torch.bfloat16)
    x = torch.randn(batch, dim, device=dev, dtype=torch.bfloat16)
    if mode.startswith("zero"):
        opt = ShardedOptimizer(model.parameters(), torch.optim.AdamW, lr=1e-4, overlap=(mode == "zero"))
        finish = None
    else:
        # replicated: fp32 master copy + AdamW state on every rank (what ZeRO shards)
        master = [p.detach().float().clone().requires_grad_(True) for p in model.parameters()]
        inner = torch.optim.AdamW(master, lr=1e-4)
        buck = ddp.GradBucketer(model)

        class _Opt:
            def step(self):
                buck.finish()
                with torch.no_grad():
                    for m, p in zip(master, model.parameters()):
                        m.grad = p.grad.float()
                    inner.step()
                    for m, p in zip(master, model.parameters()):
                        p.copy_(m)

            def zero_grad(self):
                model.zero_grad(set_to_none=False)

            def sharded_state_bytes(self):
                n = sum(m.numel() * 4 for m in master)
                for st in inner.state.values():
                    n += sum(v.numel() * v.element_size() for v in st.values() if torch.is_tensor(v))
                return n

        opt = _Opt()
        ddp.broadcast_parameters(model)
    times, tails = [], []
    for i in range(steps + 2):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        y = model(x)
        y.float().square().mean().backward()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        opt.step()
        opt.zero_grad()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if i >= 2:
            times.append(t2 - t0)
            tails.append(t2 - t1)
    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    nb = be.native_backend(None, "cuda")
    engines = {k: v[0] for k, v in nb.stats().items() if v[0] and not k.startswith(("rccl_comm", "coalesced"))}
    capped = nb.describe().split("async_capped=")[1].split(",")[0] if "async_capped=" in nb.describe() else "?"
    t = torch.tensor([statistics.median(times), statistics.median(tails)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # replicas must agree after the steps
    w = next(model.parameters()).detach().float().sum().reshape(1).cpu().double()
    ws = [torch.zeros(1, dtype=torch.float64) for _ in range(size)]
    dist.all_gather(ws, w)
    same = all(bool(v.item() == ws[0].item()) for v in ws)
    return {"mode": mode, "world": size, "params": sum(p.numel() for p in model.parameters()),
            "step_ms": round(t[0].item() * 1e3, 2), "after_backward_ms": round(t[1].item() * 1e3, 2),
            "opt_state_bytes_per_rank": opt.sharded_state_bytes(), "replicas_agree": same,
            "overlapped_buckets": getattr(opt, "overlapped", None), "engines": engines,
            "async_grid": int(os.environ.get("PDCC_IPC_ASYNC_GRID", "64")), "async_capped_launches": capped}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--dim", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--modes", default="zero,zero_nooverlap,ddp")
    ap.add_argument("--async-grids", default="64", help="comma list of PDCC_IPC_ASYNC_GRID values (0: uncapped)")
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    for rep in range(a.repeat):
        for grid in a.async_grids.split(","):
            os.environ["PDCC_IPC_ASYNC_GRID"] = grid
            for mode in a.modes.split(","):
                if grid != a.async_grids.split(",")[0] and mode == "zero_nooverlap":
                    continue  # nothing runs async without the overlap: one baseline per repeat
                res = launch(work, a.world, args=(mode, a.layers, a.dim, a.steps, a.batch), bind_device=True,
                             timeout_s=300, join_timeout_s=600)
                res[0]["repeat"] = rep
                print(json.dumps(res[0]), flush=True)


if __name__ == "__main__":
    main()
