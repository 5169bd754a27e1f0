#!/usr/bin/env python3
"""Host cost of a zero-copy IPC call when a peer is late (verdict r2, missing #3).

Two ranks share the GPU (PDCC_ALGO=ipc, 64 MiB fp32 all_reduce, zero-copy 2-shot).
Before every timed call rank 1 sleeps `--late-ms`; the line reports how long the
call took to RETURN to rank 0's host (median over trials), async_op=True and
synchronous, with the record exchange on the launcher thread (PDCC_IPC_ZC_ASYNC=1)
and inline on the caller's thread (=0, the round-2 behaviour: the caller's host
waits for its late peer). Values are checked every trial.

    python scripts/zc_async_bench.py [--late-ms 50] [--trials 7]
    python scripts/zc_async_bench.py --churn      # 40-allocation eviction churn only
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--late-ms", type=float, default=50)
    ap.add_argument("--trials", type=int, default=7)
    ap.add_argument("--churn", action="store_true")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch
    from tests import _workers as W

    if a.churn:
        env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_CACHE": "16"}
        res = launch(W.zc_churn_probe, 2, bind_device=True, timeout_s=60, env=env, join_timeout_s=300)
        print(json.dumps({"churn_allocs": 40, "ok": all(r["ok"] for r in res), "algo": res[0]["algo"],
                          "desc": res[0]["desc"][-220:], "before_barrier": res[0]["before_barrier"][-220:]}),
              flush=True)
        return
    for zc_async in ("1", "0"):
        env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_ASYNC": zc_async}
        res = launch(W.zc_async_probe, 2, args=("cuda", a.trials, 16 << 20, a.late_ms), bind_device=True,
                     timeout_s=60, env=env, join_timeout_s=300)
        r0 = res[0]
        print(json.dumps({"zc_async": int(zc_async), "bytes": 64 << 20, "peer_late_ms": a.late_ms,
                          "algo": r0["algo"], "async_return_us_rank0": round(r0["async_ret_us"], 1),
                          "sync_return_us_rank0": round(r0["sync_ret_us"], 1),
                          "correct": all(r["warm"] and r["async_ok"] and r["sync_ok"] for r in res)}), flush=True)


if __name__ == "__main__":
    main()
