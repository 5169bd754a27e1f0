"""Launcher: ``python -m pytorch_distributed_collective_communication_amd.run [opts] script.py [args]``.

Two modes:

* **self-spawning scripts** (the reference's main.py spawns its own 4 workers,
  main.py:98-108): run the script as-is with ``PDCC_TAKEOVER_GLOO=1`` and this
  package's dist-info on ``PYTHONPATH`` -- every spawned child then registers the
  ``mi355x`` backend at ``import torch`` and serves its literal
  ``init_process_group("gloo")`` (main.py:94). The script is unmodified.
* ``--nproc N``: torchrun-style, one process per rank (per GPU), with
  ``RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT`` exported, a free port
  picked (not main.py:93's fixed 29500), children's exit codes propagated and
  the survivors terminated as soon as one rank fails (main.py:107 ignores them).
  Each rank is bound to GPU ``LOCAL_RANK % visible GPUs`` (local rank ->
  hipSetDevice) when it makes its first process group, unless the script already
  chose a device (``PDCC_BIND_LOCAL_RANK=1``, parallel/backend.py).
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)


def _env(takeover: bool, extra_path: str | None = None) -> dict:
    env = dict(os.environ)
    paths = [ROOT] + ([extra_path] if extra_path else [])
    if env.get("PYTHONPATH"):
        paths.append(env["PYTHONPATH"])
    env["PYTHONPATH"] = os.pathsep.join(paths)
    if takeover:
        env["PDCC_TAKEOVER_GLOO"] = "1"
        env.setdefault("PDCC_TAKEOVER_NCCL", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return env


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m pytorch_distributed_collective_communication_amd.run")
    ap.add_argument("--nproc", type=int, default=0, help="launch N ranks (0 = the script spawns its own)")
    ap.add_argument("--no-takeover", action="store_true", help="do not map backend 'gloo' to 'mi355x'")
    ap.add_argument("--takeover-nccl", action="store_true", help="also map backend 'nccl' to 'mi355x'")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)

    env = _env(not a.no_takeover)
    if a.takeover_nccl:
        env["PDCC_TAKEOVER_NCCL"] = "1"
    cmd = [sys.executable, a.script] + a.args
    if a.nproc <= 0:
        return subprocess.call(cmd, env=env)

    from .parallel.spawn import free_port

    port = a.master_port or free_port()
    procs = []
    for r in range(a.nproc):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.nproc), MASTER_PORT=str(port),
                 LOCAL_WORLD_SIZE=str(a.nproc), PDCC_BIND_LOCAL_RANK="1")
        procs.append(subprocess.Popen(cmd, env=e))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in procs:  # one rank failed: stop the others
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs:
            q.send_signal(signal.SIGINT)
        rc = 130
    return rc


if __name__ == "__main__":
    sys.exit(main())
