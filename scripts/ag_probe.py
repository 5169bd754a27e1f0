#!/usr/bin/env python3
"""The ZeRO-style bf16 all-gather row of bench.py on W ranks sharing one GPU, engine by engine
(round 5: at W = 5, 6, 7 the full-size rehearsal's extras ran past their 240 s deadline inside
this row, while W = 3, 4, 8 finished it in well under a second).

Each engine gets its own group; rank 0 prints a line before and after every call, so a stall names
the engine and the call. `auto` races the candidates on its first call (PDCC_LOG_LEVEL=1 prints
the race).

    python scripts/ag_probe.py --world 5 --mib 2048 [--engines auto,ipc,ipc_staged,ipc_dyn]
"""
import argparse
import datetime
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, mib, engines, iters, timeout_s, verbose):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    per = (mib << 20) // 2
    ag_in = torch.full((per,), float(rank), dtype=torch.bfloat16, device=dev)
    ag_out = torch.empty(per * size, dtype=torch.bfloat16, device=dev)
    t_start = time.perf_counter()

    def say(msg):
        if rank == 0:
            print(f"[ag {time.perf_counter() - t_start:7.2f}s] {msg}", file=sys.stderr, flush=True)

    out = {}
    for engine in engines:
        g = dist.new_group(list(range(size)), timeout=datetime.timedelta(seconds=timeout_s))
        gb = be.native_backend(g, "cuda")
        gb.set_algo(engine)
        lat = []
        for i in range(iters + 1):
            ag_out.zero_()
            torch.cuda.synchronize()
            dist.barrier()
            say(f"{engine} call {i} start")
            t0 = time.perf_counter()
            dist.all_gather_into_tensor(ag_out, ag_in, group=g)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ok = torch.equal(ag_out.view(size, per)[:, -1].float().cpu(), torch.arange(size, dtype=torch.float32))
            say(f"{engine} call {i} done {dt * 1e3:.1f} ms ok={ok} engine={gb.last_algo()}")
            if verbose and rank == 0:
                d = gb.describe()
                say("  " + d[d.find(", dev"):][:1200])
            if i:
                lat.append(dt)
        t = torch.tensor([sorted(lat)[len(lat) // 2]], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out[engine] = {"p50_ms": round(t.item() * 1e3, 2), "engine": gb.last_algo(), "ok": ok}
        if engine == "auto":
            out["table"] = gb.autotune_table()
        dist.destroy_process_group(g)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=5)
    ap.add_argument("--mib", type=int, default=2048, help="bf16 input MiB per rank")
    ap.add_argument("--engines", default="auto,ipc,ipc_staged,ipc_dyn")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=60.0, help="group (and IPC spin) timeout, s")
    ap.add_argument("--env", default="", help="extra rank env, KEY=VAL[,KEY=VAL]")
    ap.add_argument("--verbose", action="store_true", help="rank 0 prints the zero-copy stats after every call")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    env = {"GPU_MAX_HW_QUEUES": "1", "PDCC_LOG_LEVEL": "1"}
    env.update(kv.split("=", 1) for kv in a.env.split(",") if kv)
    res = launch(work, a.world, args=(a.mib, a.engines.split(","), a.iters, a.timeout, a.verbose), bind_device=True,
                 timeout_s=a.timeout,
                 env=env, join_timeout_s=400)
    print(json.dumps({"world_on_one_gpu": a.world, "mib_per_rank": a.mib, **res[0]}), flush=True)


if __name__ == "__main__":
    main()
