#!/usr/bin/env python3
"""Where does the time go around a hipGraph capture of IPC collectives?
2 ranks sharing cuda:0 (IPC engine). For 4 KiB all_reduces: host issue time per
call (no sync) and synchronized per-call time, before any capture, after a
capture, and for replays. Prints one JSON line per rank."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, n_ops=16, iters=40):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel.graphs import capture

    dev = torch.device("cuda", torch.cuda.current_device())
    bufs = [torch.zeros(1024, device=dev) for _ in range(n_ops)]

    def step():
        for b in bufs:
            dist.all_reduce(b)

    def measure(tag, fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        issue = 0.0
        t0 = time.perf_counter()
        for _ in range(iters):
            a = time.perf_counter()
            fn()
            issue += time.perf_counter() - a
        torch.cuda.synchronize()
        total = time.perf_counter() - t0
        return {f"{tag}_issue_us_per_op": round(issue / iters / n_ops * 1e6, 2),
                f"{tag}_total_us_per_op": round(total / iters / n_ops * 1e6, 2)}

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    b = be.native_backend(None, "cuda")
    seen = set()

    def phases(tag):
        # PDCC_IPC_TRACE: device-side phase durations (block 0) of the calls since the last snapshot
        recs = [r for r in b.ipc_trace() if r[0] not in seen]
        seen.update(r[0] for r in recs)
        if not recs:
            return {}
        med = lambda xs: round(sorted(xs)[len(xs) // 2] / 100.0, 2)  # 100 MHz ticks -> us  # noqa: E731
        res = {f"{tag}_calls_traced": len(recs),
               f"{tag}_dev_seq_us": med([r[2] - r[1] for r in recs]),
               f"{tag}_dev_stage_us": med([r[3] - r[2] for r in recs]),
               f"{tag}_dev_barrier_us": med([r[4] - r[3] for r in recs]),
               f"{tag}_dev_reduce_us": med([r[5] - r[4] for r in recs]),
               f"{tag}_dev_total_us": med([r[7] - r[1] for r in recs])}
        st = sorted(r[1] for r in recs)
        res[f"{tag}_dev_entry_interval_us"] = med([b_ - a for a, b_ in zip(st, st[1:])])
        return res

    out = {}
    out.update(measure("eager", step))
    out.update(phases("eager"))
    g = capture(step, warmup=2)
    phases("capture")
    out.update(measure("replay", g.replay))
    out.update(phases("replay"))
    out.update(measure("eager_after", step))
    out.update(phases("eager_after"))
    return out


if __name__ == "__main__":
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    res = launch(work, 2, bind_device=True, timeout_s=60, env={"PDCC_ALGO": "ipc", "PDCC_IPC_TRACE": "8192"},
                 join_timeout_s=300)
    for r, x in enumerate(res):
        print(json.dumps({"rank": r, **x}))
