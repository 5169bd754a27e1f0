#!/usr/bin/env python3
"""The distinct-GPU test layer's phase plan (tests/test_multi_gpu.py::_plan) rehearsed with every rank on ONE
GPU: one launch per world size runs the phases in plan order (the default group re-made per phase), skipping
those that need one rank per device (RCCL forced, communicator churn, device binding). Prints each phase's
verdict: ok, a failed check, or the phase's error -- the re-made-group sequence the 8-GPU node will run.

    python scripts/plan_rehearsal.py [--world 2 4]
"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NEEDS_DISTINCT = ("group_churn", "device_id", "split", "p2p", "list_all_gather", "crosscheck")


def verdict(v):
    if isinstance(v, dict) and "__error__" in v:
        return "error: " + v["__error__"][:300]
    if isinstance(v, dict):
        if "all_ok" in v:
            return "ok" if v["all_ok"] else "failed: " + json.dumps(
                {k: c for k, c in v.get("checks", {}).items() if not c.get("ok")})[:1500]
        bad = [k for k, x in v.items() if x is False]
        return "ok" if not bad else "failed: " + ", ".join(bad)[:300]
    if isinstance(v, list) and all(isinstance(x, bool) for x in v):
        return "ok" if all(v) else f"failed: {v}"
    return "ran"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="*", default=[2, 4])
    ap.add_argument("--only", nargs="*", default=None, help="phase keys to run (default: every one)")
    ap.add_argument("--hwq", default="1", help="GPU_MAX_HW_QUEUES for 5+ ranks ('' = the runtime's default)")
    a = ap.parse_args()
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch
    from tests import _workers as W
    from tests.test_multi_gpu import _plan

    for w in a.world:
        d = tempfile.mkdtemp()
        plan = [p for p in _plan(w, d) if p[3].get("PDCC_ALGO") != "rccl" and not p[0].startswith(NEEDS_DISTINCT)
                and (a.only is None or p[0] in a.only)]
        # (5+ ranks on one GPU: one hardware queue each, as the shared-GPU tests run them)
        env = {"GPU_MAX_HW_QUEUES": a.hwq} if w >= 5 and a.hwq else {}
        res = launch(W.distinct_suite, w, args=("cuda", tuple(plan), d), bind_device=True, timeout_s=120,
                     join_timeout_s=900, env=env)
        for key, *_ in plan:
            print(json.dumps({"world": w, "phase": key, "per_rank": [verdict(r[key]) for r in res]}), flush=True)


if __name__ == "__main__":
    main()
