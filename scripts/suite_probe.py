#!/usr/bin/env python3
"""Isolate a failing bulk all_reduce in a group made after another group of the same ranks ran small
(LL) collectives (tests/_workers.py regroup_probe / distinct_suite), ranks sharing one GPU."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_collective_communication_amd.parallel.spawn import launch  # noqa: E402
from tests import _workers as W  # noqa: E402


def one(name, fn, args, env):
    try:
        r = launch(fn, 2, args=args, bind_device=True, timeout_s=60, env=env, join_timeout_s=200)
    except Exception as e:  # noqa: BLE001
        r = str(e)[:600]
    print(json.dumps({name: r}), flush=True)


def falses(r):
    if isinstance(r, str):
        return r
    out = []
    for got in r:
        row = {}
        for k, v in got.items():
            if isinstance(v, dict):
                row[k] = v.get("__error__") or [n for n, ok in v.items() if ok is not True]
        out.append(row)
    return out


def suite(name, phases):
    d = tempfile.mkdtemp()
    try:
        r = launch(W.distinct_suite, 2, args=("cuda", phases, d), bind_device=True, timeout_s=120, join_timeout_s=300)
    except Exception as e:  # noqa: BLE001
        r = str(e)[:600]
    print(json.dumps({name: falses(r)}), flush=True)


def main():
    zc_env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_CACHE": "4", "PDCC_IPC_1SHOT_MAX": "256K", "PDCC_IPC_MAX_STAGING": "8M",
              "PDCC_IPC_VA_LOG": "1"}
    golden = ("golden/ipc", "golden", ("cuda",), {"PDCC_ALGO": "ipc"})
    diag = ("diag", "zc_reuse_diag", ("cuda",), zc_env)
    for i in range(8):
        d = tempfile.mkdtemp()
        r = launch(W.distinct_suite, 2, args=("cuda", (golden, diag), d), bind_device=True, timeout_s=120,
                   join_timeout_s=300, env={"PDCC_IPC_VA_LOG": "1"})
        print(json.dumps({f"#{i}": [x["diag"] for x in r]}), flush=True)
        if any(c[0] for x in r for c in x["diag"]["calls"]):
            break


if __name__ == "__main__":
    main()
