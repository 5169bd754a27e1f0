#!/usr/bin/env python3
"""Per-call host overhead of a GPU collective, world of 1 on one GPU.

    python scripts/host_overhead.py mi355x   # our backend, RCCL forced on a 1-rank comm
    python scripts/host_overhead.py nccl     # torch's ProcessGroupNCCL (same RCCL underneath)

Reports the host-side enqueue time per all_reduce (4 B) and the end-to-end
time per call including the GPU (both averaged over 2000 calls), for the
synchronous form and for ``async_op=True`` followed by ``Work.wait()`` (which
crosses to the backend's comm stream and back).
"""
import datetime
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    backend = sys.argv[1] if len(sys.argv) > 1 else "mi355x"
    os.environ["PDCC_WORLD1_LOCAL"] = "0"
    import torch
    import torch.distributed as dist

    import pytorch_distributed_collective_communication_amd  # noqa: F401  (registers mi355x)
    from pytorch_distributed_collective_communication_amd.parallel.spawn import free_port

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(free_port())
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=0, world_size=1, timeout=datetime.timedelta(seconds=60))
    t = torch.ones(1, device="cuda")
    for _ in range(50):
        dist.all_reduce(t)
    torch.cuda.synchronize()
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        dist.all_reduce(t)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    t3 = time.perf_counter()
    for _ in range(n):
        dist.all_reduce(t, async_op=True).wait()
    t4 = time.perf_counter()
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    print(json.dumps({"backend": backend, "stream": os.environ.get("PDCC_STREAM", "auto"),
                      "enqueue_us": round((t1 - t0) / n * 1e6, 2),
                      "end_to_end_us": round((t2 - t0) / n * 1e6, 2),
                      "async_wait_enqueue_us": round((t4 - t3) / n * 1e6, 2),
                      "async_wait_end_to_end_us": round((t5 - t3) / n * 1e6, 2)}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
