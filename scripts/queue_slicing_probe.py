#!/usr/bin/env python3
"""Why the W=8 shared-GPU bench rehearsal's extras sit at ~56 ms per op (verdict r4 Next #4).

W ranks share ONE GPU (a rehearsal only: the driver runs one rank per GPU). Each rank times
all_reduces of 4 B (LL: wall time only, the LL kernels are not traced), 1 MiB and 64 MiB
(2-shot: PDCC_IPC_TRACE device stamps) twice: on a fresh group, and again after the bench's
conformance pass (which adds async collectives -- a comm stream, i.e. another hardware queue
per process -- plus coalesced, capped-grid and raced calls).

For every traced call, matched across ranks by block 0's call number (header word 0), the
device clock (s_memrealtime, 100 MHz, one clock for every process on the GPU) splits the
wall time into
  * start_skew_us:  last rank's kernel entry - first rank's kernel entry (a rank's kernel
                    waiting for its queue to be scheduled: the peers spin in the arrival barrier)
  * body_us:        last rank's exit - last rank's entry (the protocol itself).
Time-slicing of hardware queues shows as a start skew of a scheduling quantum at unchanged
bodies. ``--queues 1`` runs every rank with GPU_MAX_HW_QUEUES=1 (all its streams on one
hardware queue), which keeps W=8 processes within the queues the GPU maps at once.

    python scripts/queue_slicing_probe.py --world 8 [--queues 1] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be
    from pytorch_distributed_collective_communication_amd.utils import conformance

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    out = {"rank": rank}

    def measure(tag):
        res = {}
        for nb in (4, 1 << 20, 64 << 20):
            x = torch.ones(max(1, nb // 4), device=dev)
            for _ in range(2):
                dist.all_reduce(x)
            walls = []
            for _ in range(iters):
                x.fill_(1.0)
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                dist.all_reduce(x)
                torch.cuda.synchronize()
                walls.append(time.perf_counter() - t0)
            ok = bool(torch.all(x == size).item())
            row = {"engine": b.last_algo(), "ok": ok, "wall_us": round(statistics.median(walls) * 1e6, 1)}
            if nb >= 1 << 20:
                recs = sorted((r for r in b.ipc_trace() if r[1] and r[7]), key=lambda r: r[0])[-iters:]
                mine = {int(r[0]): (int(r[1]), int(r[7])) for r in recs}
                allr = [None] * size
                dist.all_gather_object(allr, mine)
                skew, body = [], []
                for seq in mine:
                    if all(seq in a for a in allr):
                        ent = [a[seq][0] for a in allr]
                        ext = [a[seq][1] for a in allr]
                        skew.append((max(ent) - min(ent)) / 100.0)
                        body.append((max(ext) - max(ent)) / 100.0)
                row.update(calls=len(skew), start_skew_us=round(statistics.median(skew), 1) if skew else None,
                           start_skew_max_us=round(max(skew), 1) if skew else None,
                           body_us=round(statistics.median(body), 1) if body else None)
            res[f"{nb}B"] = row
            del x
        out[tag] = res

    measure("fresh")
    t0 = time.time()
    conf = conformance.run(rank, size, dev, deadline_s=120.0, max_bytes=64 << 20)
    out["conformance"] = {"all_ok": conf["all_ok"], "passed": conf["passed"], "failed": conf["failed"],
                          "elapsed_s": round(time.time() - t0, 1)}
    measure("after_conformance")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--queues", type=int, default=0, help="GPU_MAX_HW_QUEUES per rank (0: the runtime default)")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    env = {"PDCC_IPC_TRACE": "64", "PDCC_ALGO": "ipc"}
    if a.queues:
        env["GPU_MAX_HW_QUEUES"] = str(a.queues)
    res = launch(work, a.world, args=(a.iters,), bind_device=True, timeout_s=120, env=env, join_timeout_s=500)
    r0 = res[0]
    print(json.dumps({"world_on_one_gpu": a.world, "gpu_max_hw_queues": a.queues or "default",
                      "fresh": r0["fresh"], "after_conformance": r0["after_conformance"],
                      "conformance": r0["conformance"]}), flush=True)


if __name__ == "__main__":
    main()
