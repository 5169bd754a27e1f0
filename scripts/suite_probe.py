#!/usr/bin/env python3
"""Re-made groups on a shared GPU: runs tests/_workers.py::distinct_suite with a sequence of phases (each
re-makes the default group) and reports the last phase's diagnostics -- `bulk_pre_diag` (the fresh input
checked on the host before the call, then the result), `zc_reuse_diag`, `regroup_probe`. The probes behind
profiles/r6/regroup/README.md; edit main() for other phase sequences.

    python scripts/suite_probe.py        (2 ranks on GPU 0)
"""
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


def raw(name, phases, env=None):
    d = tempfile.mkdtemp()
    try:
        r = launch(W.distinct_suite, 2, args=("cuda", phases, d), bind_device=True, timeout_s=120, join_timeout_s=300,
                   env=env or {})
        r = [x.get("diag") for x in r]
    except Exception as e:  # noqa: BLE001
        r = str(e)[:600]
    print(json.dumps({name: r}), flush=True)


def main():
    ph = {"golden": ("golden/ipc", "golden", ("cuda",), {"PDCC_ALGO": "ipc"}),
          "ll": ("ll", "ll_probe", ("cuda",), {"PDCC_ALGO": "ipc"}),
          "diag": ("diag", "bulk_pre_diag", ("cuda",), {"PDCC_ALGO": "ipc"}),
          "diag_host": ("diag", "bulk_pre_diag", ("cuda",), {"PDCC_ALGO": "host"})}
    for names in (("ll", "diag"), ("golden", "diag"), ("golden", "ll", "diag")):
        for i in range(2):
            raw(" > ".join(names) + f" #{i}", tuple(ph[n] for n in names))


if __name__ == "__main__":
    main()
