#!/usr/bin/env python3
"""Small all_gather (LL) vs small all_reduce, ranks sharing one GPU: per-call wall time of back-to-back
calls, host time of the Python call, and the backend's per-stage host profile, for 4 B and 64 KiB per rank
(flat output and list output).

    python scripts/ag_small_probe.py [--world 4] [--calls 500]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, calls):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    out = {}
    for nbytes in (4, 64 << 10):
        n = max(1, nbytes // 4)
        x = torch.full((n,), float(rank + 1), device=dev)
        flat = torch.empty(n * size, device=dev)
        lst = [torch.empty(n, device=dev) for _ in range(size)]
        cases = {"all_reduce": lambda: dist.all_reduce(x),
                 "ag_flat": lambda: dist.all_gather_into_tensor(flat, x),
                 "ag_list": lambda: dist.all_gather(lst, x)}
        for name, fn in cases.items():
            for _ in range(50):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            b.set_host_profile(True)
            host = []
            t0 = time.perf_counter()
            for _ in range(calls):
                h0 = time.perf_counter()
                fn()
                host.append(time.perf_counter() - h0)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / calls
            prof = b.host_profile()
            b.set_host_profile(False)
            t = torch.tensor([wall], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            out[f"{name}/{nbytes}B"] = {
                "algo": b.last_algo(), "per_call_us": round(t.item() * 1e6, 2),
                "py_call_us": round(statistics.median(host) * 1e6, 2),
                "stages_us": {s: round(tot / max(1, k), 2) for s, (k, tot) in prof.items() if tot > 0}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--calls", type=int, default=500)
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    env = {"PDCC_ALGO": "ipc", "PDCC_HOST_PROF": "1"}
    if a.world >= 5:
        env["GPU_MAX_HW_QUEUES"] = "1"
    r = launch(work, a.world, args=(a.calls,), bind_device=True, timeout_s=120, env=env, join_timeout_s=300)
    for k, v in r[0].items():
        print(json.dumps({"world": a.world, "case": k, **v}), flush=True)


if __name__ == "__main__":
    main()
