#!/usr/bin/env python3
"""Cost of the reference's group pattern on the RCCL path: main.py builds a
fresh ``new_group(range(size))`` in every demo (main.py:11,21,31,46,63,75).
World of 1 with PDCC_WORLD1_LOCAL=0 (RCCL refuses two ranks on one GPU, so a
1-GPU box can only time 1-rank communicators), 6 groups per mode; prints one
JSON line per mode with the per-group wall time of new_group + first
all_reduce and the communicator setup time."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch
    from tests import _workers as W

    for mode in ("init", "split", "share"):
        env = {"PDCC_WORLD1_LOCAL": "0", "PDCC_RCCL_GROUP_COMM": mode}
        res = launch(W.group_churn, 1, args=("cuda", 6), bind_device=True, env=env, timeout_s=120)[0]
        res["mode"] = mode
        res["sum_wall_ms_after_first"] = round(sum(g["wall_ms"] for g in res["groups"]), 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
