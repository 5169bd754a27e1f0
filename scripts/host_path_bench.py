#!/usr/bin/env python3
"""Where the host time of one small GPU all_reduce goes (verdict r2 weak #6).

Two ranks share the GPU (PDCC_ALGO=ipc). Per case, `--calls` back-to-back
dist.all_reduce calls with the backend's stage profiler on (PDCC_HOST_PROF):
  py_call_us   -- host time of the Python call (dist.all_reduce returns), median
  per_call_us  -- wall time per call of the back-to-back loop incl. the GPU (max over ranks)
  stages_us    -- mean per call of each C++ stage (before_op, dev_state, choose, pre,
                  enqueue, work, record), and `c10d_python` = py_call - sum(stages)
Cases: 4 B (LL kernel), 64 KiB (LL), 1 / 4 / 16 MiB sync and 4 MiB async (zero-copy: gated
launch + exchange job on the IPC launcher thread; `xchg` = that thread's mean queue wait and
exchange time per job).

    python scripts/host_path_bench.py [--calls 2000]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, calls, trace=False):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    out = {}
    seen_seq = set()
    import re

    cases = (("4B", 4, False), ("64KiB", 64 << 10, False), ("1MiB", 1 << 20, False), ("4MiB", 4 << 20, False),
             ("4MiB_async", 4 << 20, True), ("16MiB", 16 << 20, False))
    for name, nbytes, async_op in cases:
        x = torch.full((max(1, nbytes // 4),), 1.0, device=dev)
        for _ in range(50):
            w = dist.all_reduce(x, async_op=async_op)
        torch.cuda.synchronize()
        dist.barrier()
        b.set_host_profile(True)
        host = []
        k = calls if nbytes <= (64 << 10) else calls // 10
        t0 = time.perf_counter()
        for _ in range(k):
            h0 = time.perf_counter()
            w = dist.all_reduce(x, async_op=async_op)
            host.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / k
        algo = b.last_algo()
        prof = b.host_profile()
        b.set_host_profile(False)
        stages = {s: (tot / max(1, n)) for s, (n, tot) in prof.items()}
        py = statistics.median(host) * 1e6
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out_trace = None
        out[name] = {"algo": algo, "py_call_us": round(py, 2), "per_call_us": round(t.item() * 1e6, 2),
                     "stages_us": {s: round(v, 2) for s, v in stages.items()},
                     "c10d_python_us": round(py - sum(stages.values()), 2)}
        if trace:  # device phase trace of block 0 (PDCC_IPC_TRACE, 100 MHz ticks) of this case's IPC calls
            recs = [r for r in b.ipc_trace() if r[0] not in seen_seq and r[1] and r[7]]
            seen_seq.update(r[0] for r in recs)
            if recs:
                med = lambda xs: round(statistics.median(xs) / 100.0, 2)  # noqa: E731
                gated = [r for r in recs if r[3] and r[2] and r[3] <= r[2]]  # [3] = gate passed (before arrival)
                out_trace = {"calls": len(recs), "entry_to_arrival_us": med([r[2] - r[1] for r in recs if r[2]]),
                             "gated_calls": len(gated),
                             "gate_wait_us": med([r[3] - r[1] for r in gated]) if gated else None,
                             # device-side exchange phases (block 0): records in / lookup / votes / published
                             "zx_records_us": med([r[8] - r[1] for r in gated if r[8]]) if gated else None,
                             "zx_lookup_us": med([r[9] - r[8] for r in gated if r[9]]) if gated else None,
                             "zx_vote_us": med([r[10] - r[9] for r in gated if r[10]]) if gated else None,
                             "zx_publish_us": med([r[11] - r[10] for r in gated if r[11]]) if gated else None,
                             "arrival_to_exit_us": med([r[7] - r[2] for r in recs if r[2]]),
                             "kernel_us": med([r[7] - r[1] for r in recs])}
        m = re.search(r"launcher_jobs=(\d+).*?xchg_wait_us=(\d+), xchg_us=(\d+), xchg_gather_us=(\d+), "
                      r"xchg_depth_x10=(\d+)", b.describe())
        if m:  # zero-copy exchange thread, cumulative means (jobs so far)
            out[name]["xchg"] = {"jobs": int(m.group(1)), "wait_us": int(m.group(2)), "run_us": int(m.group(3)),
                                 "gather_us": int(m.group(4)), "queue_depth": int(m.group(5)) / 10}
        if out_trace:
            out[name]["device_trace"] = out_trace
        x.fill_(1.0)
        dist.all_reduce(x)
        out[name]["correct"] = bool(torch.all(x == size).item())
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--trace", action="store_true", help="PDCC_IPC_TRACE: device phase times of block 0")
    ap.add_argument("--env", nargs="*", default=[], help="extra KEY=VALUE for the ranks (e.g. PDCC_IPC_ZC_ASYNC=0)")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    env = {"PDCC_ALGO": "ipc"}
    env.update(kv.split("=", 1) for kv in a.env)
    if a.trace:
        env["PDCC_IPC_TRACE"] = "65536"
    res = launch(work, a.world, args=(a.calls, a.trace), bind_device=True, timeout_s=60, env=env,
                 join_timeout_s=300)
    for name, r in res[0].items():
        print(json.dumps({"world_on_one_gpu": a.world, "case": name, **r}), flush=True)
