#!/usr/bin/env python3
"""Debug harness: run one tests/_workers.py worker on W ranks sharing the GPU with
PDCC_LOG_LEVEL (default 3: every collective + IPC launcher jobs) and a faulthandler
dump of every rank's Python stack after --dump-s seconds.

    python scripts/zc_debug.py zero_copy --world 3 --env PDCC_ALGO=ipc PDCC_IPC_ZC_CACHE=4
"""
import argparse
import faulthandler
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _wrapped(rank, size, name, dump_s):
    faulthandler.dump_traceback_later(dump_s, exit=True)
    from tests import _workers as W

    return getattr(W, name)(rank, size)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("worker")
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--dump-s", type=float, default=45)
    ap.add_argument("--env", nargs="*", default=[])
    a = ap.parse_args()
    env = dict(kv.split("=", 1) for kv in a.env)
    env.setdefault("PDCC_LOG_LEVEL", "3")
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    res = launch(_wrapped, a.world, args=(a.worker, a.dump_s), bind_device=True, timeout_s=60, env=env,
                 join_timeout_s=a.dump_s + 30)
    print(res)


if __name__ == "__main__":
    main()
