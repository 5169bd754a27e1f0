#!/usr/bin/env python3
"""Eager issue vs hipGraph replay of a launch-bound collective step: 16 small
all_reduces (4 KiB each), captured with parallel.graphs.capture.

    python scripts/graph_bench.py                      # 2 ranks sharing cuda:0, IPC kernels
    GRAPH_BENCH_MODE=rccl1 python scripts/graph_bench.py   # 1 rank, RCCL forced (PDCC_WORLD1_LOCAL=0)

On one GPU the IPC "peers" are local HBM, so this measures the host launch and
protocol cost per step -- exactly what a graph replay removes. The two ranks
share the GPU, so each process is held to one hardware queue
(GPU_MAX_HW_QUEUES=1): the capture's side stream would otherwise give each
process more queues than the GPU maps at once, and the hardware scheduler then
time-slices the two processes' queues -- the IPC kernels of one rank wait a
slice (~40 us) for the peer's (profiles/graph_probe_r2.jsonl vs
graph_probe_q1_r2.jsonl). One process per GPU never shares a GPU's queues.
Prints one JSON line.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, n_ops, numel, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel.graphs import capture

    dev = torch.device("cuda", torch.cuda.current_device())
    bufs = [torch.zeros(numel, device=dev) for _ in range(n_ops)]

    def step():
        for b in bufs:
            dist.all_reduce(b)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e6

    eager = timed(step)
    g = capture(step, warmup=2)
    replay = timed(g.replay)
    # eager again after the capture: the IPC kernels now take their sequence numbers from the
    # device counter too (graph mode), which isolates that cost from the graph launch itself
    eager_dev_seq = timed(step)
    for b in bufs:
        b.fill_(float(rank + 1))
    g.replay()
    torch.cuda.synchronize()
    ok = all(bool(torch.all(b == size * (size + 1) / 2).item()) for b in bufs)
    return {"eager_us_per_step": round(eager, 1), "replay_us_per_step": round(replay, 1),
            "eager_us_per_op": round(eager / n_ops, 2), "replay_us_per_op": round(replay / n_ops, 2),
            "eager_after_capture_us_per_op": round(eager_dev_seq / n_ops, 2), "correct": ok}


if __name__ == "__main__":
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    mode = os.environ.get("GRAPH_BENCH_MODE", "ipc2")
    world, env = (1, {"PDCC_WORLD1_LOCAL": "0"}) if mode == "rccl1" else (2, {"PDCC_ALGO": "ipc",
                                                                          "GPU_MAX_HW_QUEUES": "1"})
    out = launch(work, world, args=(16, 1024, 50), bind_device=True, timeout_s=60, env=env, join_timeout_s=300)
    print(json.dumps({"mode": mode, "ranks_on_one_gpu": world, "ops_per_step": 16, "bytes_per_op": 4096,
                      "per_rank": out}))
