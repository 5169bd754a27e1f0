#!/usr/bin/env python3
"""Where the time of one big IPC all_reduce goes (verdict r3 Next #7): device phase trace
of the 2-shot all_reduce (zero-copy and staged) with W ranks sharing ONE GPU, next to K1
(the same 2-source reduce the pull phase does) at the same workgroup budget.

PDCC_IPC_TRACE records block 0's s_memrealtime stamps (100 MHz) per launch
(kern::kTraceWords): [1] entry, [2] arrival barrier, [3] gate passed / staged,
[4] data barrier, [5] phase 1 (reduce own tiles) done, [6] second barrier, [7] exit;
the dynamic protocols add block 0's totals: [16] claim waits, [17] ready publishing,
[18] ready waits, [19] departure, [20] items, [21] phase-1 items, [22] departed last,
[23] epoch read.
Per phase the median over the timed calls, in microseconds, plus the HBM traffic
model of each protocol and the rates it implies:

* zero-copy 2-shot, per rank: phase 1 reads W own-tile slices (one per rank's tensor)
  and writes S/W in place; phase 2 copies the (W-1)/W peer-owned part:
  reads S(1 + (W-1)/W) ... writes S; W ranks share the GPU's HBM.
* staged: + the staging copy (read S, write S) and phase 2 from staging.

Ranks sharing one GPU run each IPC grid at 256 / W workgroups (co-residency: every
block spins on its peer block), so K1 is timed at the same total workgroup count.

    python scripts/ipc_phase_trace.py [--world 2] [--mib 256] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def work(rank, size, mib, iters):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd import ops
    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dev = torch.device("cuda", torch.cuda.current_device())
    b = be.native_backend(None, "cuda")
    n = (mib << 20) // 4
    x = torch.full((n,), float(rank + 1), device=dev)
    for _ in range(3):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    dist.barrier()
    walls = []
    for _ in range(iters):
        x.fill_(float(rank + 1))
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        dist.all_reduce(x)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    ok = bool(torch.all(x == size * (size + 1) / 2).item())
    recs = [r for r in b.ipc_trace() if r[1] and r[7]][-iters:]

    def ph(a, c):
        v = [(r[c] - r[a]) / 100.0 for r in recs if r[a] and r[c] and r[c] >= r[a]]
        return round(statistics.median(v), 1) if v else None

    phases = {"entry_to_arrival": ph(1, 2), "arrival_to_data_barrier": ph(2, 4), "stage_or_gate": ph(2, 3),
              "phase1_reduce": ph(4, 5), "barrier2": ph(5, 6), "phase2_gather": ph(6, 7), "kernel_total": ph(1, 7),
              # block 0's device-side buffer exchange of a gated zero-copy launch (words 8-11)
              "zx_records_in": ph(1, 8), "zx_lookup": ph(8, 9), "zx_votes_in": ph(9, 10), "zx_published": ph(10, 11),
              "zx_to_arrival": ph(11, 2), "zx_to_args_staged": ph(11, 3), "args_staged_to_arrival": ph(3, 2),
              # inside: call number taken, every wave drained, flags stored, every peer's flag seen
              "block_seq": ph(3, 12), "barrier_drain": ph(12, 13), "barrier_store": ph(13, 14),
              "barrier_poll": ph(14, 15), "barrier_acquire": ph(15, 2)}
    # dynamic protocols (--algo ipc_dyn): block 0's totals per call (words 16-23)

    def tot(k, scale=100.0):
        v = [r[k] / scale for r in recs if len(r) > 23]
        return round(statistics.median(v), 1) if v and any(v) else None

    phases.update({"dyn_claim_wait": tot(16), "dyn_ready_publish": tot(17), "dyn_ready_wait": tot(18),
                   "dyn_departure": tot(19), "dyn_items_block0": tot(20, 1.0), "dyn_phase1_items_block0": tot(21, 1.0),
                   "dyn_block0_last": tot(22, 1.0), "dyn_epoch_read": tot(23)})
    out = {"rank": rank, "engine": b.last_algo(), "correct": ok, "wall_us": round(statistics.median(walls) * 1e6, 1),
           "phases_us": phases, "records": len(recs), "blocks_us": block_spread(recs)}
    # K1 at the same total workgroup budget: rank 0 alone, the others wait
    dist.barrier()
    if rank == 0:
        s = [torch.rand(n // size, device=dev) for _ in range(2)]
        o = torch.empty(n // size, device=dev)
        k1 = {}
        for blocks in (256 // size, 256, 0):
            for _ in range(2):
                ops.reduce_nway(s, out=o, impl="lds_ntl", max_blocks=blocks)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                ops.reduce_nway(s, out=o, impl="lds_ntl", max_blocks=blocks)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            k1[f"k1_2src_{blocks or 'default'}wg_GBps"] = round(3 * o.numel() * 4 / dt / 1e9, 1)
        out["k1"] = k1
    dist.barrier()
    return out


HDR, NB = 24, 256  # kern::kTraceWords, kern::kTraceBlocks


def block_spread(recs):
    """Every block against block 0 (per-block stamps after the header, measured from block
    0's entry): median over calls of the median / slowest block's phase-1 end and exit."""
    p1_med, p1_max, ex_med, ex_max, n = [], [], [], [], 0
    for r in recs:
        if len(r) < HDR + 2 * NB:
            return None
        t0 = r[1]
        p1 = [(x - t0) / 100.0 for x in r[HDR:HDR + NB] if x >= t0]
        ex = [(x - t0) / 100.0 for x in r[HDR + NB:HDR + 2 * NB] if x >= t0]
        if not ex:
            continue
        n = max(n, len(ex))
        ex_med.append(statistics.median(ex))
        ex_max.append(max(ex))
        if p1:
            p1_med.append(statistics.median(p1))
            p1_max.append(max(p1))

    def med(v):
        return round(statistics.median(v), 1) if v else None

    return {"blocks": n, "phase1_done_median_block": med(p1_med), "phase1_done_slowest_block": med(p1_max),
            "exit_median_block": med(ex_med), "exit_slowest_block": med(ex_max)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--modes", default="zc,staged")
    ap.add_argument("--algo", default="ipc", help="PDCC_ALGO of the traced calls (ipc, ipc_dyn, ...)")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    S = a.mib << 20
    W = a.world
    for mode in a.modes.split(","):
        env = {"PDCC_ALGO": a.algo, "PDCC_IPC_TRACE": "64", "PDCC_IPC_ZC": "0" if mode == "staged" else "1",
               "PDCC_AUTOTUNE": "0"}
        res = launch(work, W, args=(a.mib, a.iters), bind_device=True, timeout_s=120, env=env, join_timeout_s=400)
        # HBM bytes per call, all ranks together (one GPU): reads / writes
        if mode == "zc":
            rd, wr = W * S * (1 + (W - 1) / W), W * S
        else:
            rd, wr = W * S * (2 + (W - 1) / W), W * S * (1 + 1 + 1 / W)
        # the trace is per launch: a zero-copy call above 256 MiB runs as launches of at most 256 MiB
        # (launcher.cpp kGateChunk), so the rates below are per launch
        per = min(S, 256 << 20) / S if mode == "zc" else 1.0
        for r in res:
            r.update(mode=mode, algo=a.algo, world_on_one_gpu=W, bytes=S, hbm_read_bytes=int(rd), hbm_write_bytes=int(wr),
                     launch_fraction=per)
            kt = r["phases_us"]["kernel_total"]
            if kt:
                r["hbm_TBps_kernel"] = round(per * (rd + wr) / (kt * 1e-6) / 1e12, 2)
            p1 = r["phases_us"]["phase1_reduce"]
            if p1:  # phase 1 alone: every rank reads W slices of S/W and writes S/W
                r["hbm_TBps_phase1"] = round(per * W * (S + S / W) / (p1 * 1e-6) / 1e12, 2)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
