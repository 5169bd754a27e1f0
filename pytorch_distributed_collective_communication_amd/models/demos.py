"""The tutorial's workloads as reusable functions (reference main.py:9-87).

Each ``(rank, size, device="cpu") -> value`` function runs one collective the
way the reference demonstrates it -- a fresh ``new_group`` over all ranks, the
same tensors and roots -- prints the same ``[rank] data = ...`` line and also
returns the result so tests and notebooks can check it.

Golden outputs (README.md of the reference, 4 ranks): reduce -> 4.0 at rank 0;
all_reduce -> 4.0 everywhere; scatter -> rank r gets r+1; gather -> rank 0 gets
[0., 1., 2., 3.]; all_gather -> everybody gets [0., 1., 2., 3.]; broadcast ->
everybody gets tensor([0.]). Non-root ``reduce`` buffers keep their input here
(the reference's 3/2/1 are Gloo leftovers).

CLI: ``python -m pytorch_distributed_collective_communication_amd.models.demos
--demo scatter --world 4 [--device cuda]``.
"""
from __future__ import annotations

import argparse

import torch
import torch.distributed as dist


def _dev(device):
    return torch.device("cpu") if device == "cpu" else torch.device("cuda", torch.cuda.current_device())


def hello_world(rank: int, size: int, device: str = "cpu"):
    msg = f"[{rank}] say hi!"
    print(msg, flush=True)
    return msg


def do_reduce(rank: int, size: int, device: str = "cpu", op=dist.ReduceOp.SUM):
    group = dist.new_group(list(range(size)))
    t = torch.ones(1, device=_dev(device))
    dist.reduce(t, dst=0, op=op, group=group)  # only rank 0 holds the result
    print(f"[{rank}] data = {t[0]}", flush=True)
    return t.item()


def do_all_reduce(rank: int, size: int, device: str = "cpu", op=dist.ReduceOp.SUM):
    group = dist.new_group(list(range(size)))
    t = torch.ones(1, device=_dev(device))
    dist.all_reduce(t, op=op, group=group)
    print(f"[{rank}] data = {t[0]}", flush=True)
    return t.item()


def do_scatter(rank: int, size: int, device: str = "cpu"):
    d = _dev(device)
    group = dist.new_group(list(range(size)))
    t = torch.empty(1, device=d)
    chunks = [torch.tensor([r + 1.0], device=d) for r in range(size)] if rank == 0 else []
    dist.scatter(t, scatter_list=chunks, src=0, group=group)
    print(f"[{rank}] data = {t[0]}", flush=True)
    return t.item()


def do_gather(rank: int, size: int, device: str = "cpu"):
    d = _dev(device)
    group = dist.new_group(list(range(size)))
    t = torch.tensor([float(rank)], device=d)
    bucket = [torch.empty(1, device=d) for _ in range(size)] if rank == 0 else []
    dist.gather(t, gather_list=bucket, dst=0, group=group)
    if rank == 0:
        print(f"[{rank}] data = {[b.cpu() for b in bucket]}", flush=True)
        return [b.item() for b in bucket]
    return None


def do_all_gather(rank: int, size: int, device: str = "cpu"):
    d = _dev(device)
    group = dist.new_group(list(range(size)))
    t = torch.tensor([float(rank)], device=d)
    bucket = [torch.empty(1, device=d) for _ in range(size)]
    dist.all_gather(bucket, t, group=group)
    print(f"[{rank}] data = {[b.cpu() for b in bucket]}", flush=True)
    return [b.item() for b in bucket]


def do_broadcast(rank: int, size: int, device: str = "cpu"):
    d = _dev(device)
    group = dist.new_group(list(range(size)))
    t = torch.tensor([0.0], device=d) if rank == 0 else torch.empty(1, device=d)
    dist.broadcast(t, src=0, group=group)
    print(f"[{rank}] data = {t.cpu()}", flush=True)
    return t.item()


DEMOS = {
    "hello_world": hello_world,
    "reduce": do_reduce,
    "all_reduce": do_all_reduce,
    "scatter": do_scatter,
    "gather": do_gather,
    "all_gather": do_all_gather,
    "broadcast": do_broadcast,
}


def golden(name: str, rank: int, size: int):
    """Expected return value of ``DEMOS[name]`` on ``rank``."""
    return {
        "hello_world": f"[{rank}] say hi!",
        "reduce": float(size) if rank == 0 else 1.0,
        "all_reduce": float(size),
        "scatter": rank + 1.0,
        "gather": [float(r) for r in range(size)] if rank == 0 else None,
        "all_gather": [float(r) for r in range(size)],
        "broadcast": 0.0,
    }[name]


def main(argv=None):
    from ..parallel.spawn import launch

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--demo", default="scatter", choices=sorted(DEMOS))
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
    a = ap.parse_args(argv)
    res = launch(DEMOS[a.demo], a.world, args=(a.device,), bind_device=a.device == "cuda")
    bad = [r for r, v in enumerate(res) if v != golden(a.demo, r, a.world)]
    if bad:
        raise SystemExit(f"golden mismatch on ranks {bad}: {res}")


if __name__ == "__main__":
    main()
