"""Process launching: the reference's ``init_process`` + ``mp.Process`` loop
(reference main.py:90-108), made robust.

Differences from the reference (all deliberate):

* the rendezvous port is picked free instead of the fixed 29500 (main.py:93),
  so concurrent runs do not collide;
* child exit codes are checked (main.py:107-108 ignores them): a failing rank
  raises in the parent and the surviving ranks are terminated;
* each rank's return value is sent back to the parent (tests use this);
* ``LOCAL_RANK`` is exported and, when GPUs are visible, each rank is bound to
  ``cuda:LOCAL_RANK`` (one process per GPU).
"""
from __future__ import annotations

import os
import socket
import traceback
from typing import Any, Callable, Sequence

import torch.multiprocessing as mp

from .backend import BACKEND_NAME


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def init_process(
    rank: int,
    size: int,
    fn: Callable[..., Any],
    backend: str = BACKEND_NAME,
    port: int | None = None,
    args: Sequence[Any] = (),
    bind_device: bool = False,
    timeout_s: float | None = None,
):
    """Same contract as the reference's ``init_process(rank, size, fn, backend)``:
    set up env:// rendezvous, ``init_process_group``, then ``fn(rank, size, *args)``."""
    import datetime

    import torch
    import torch.distributed as dist

    from .. import register

    register()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if port is not None:
        os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("MASTER_PORT", "29500")
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(size)
    os.environ.setdefault("LOCAL_RANK", str(rank))
    if bind_device and torch.cuda.device_count() > 0:
        # PDCC_SPAWN_DEVICE=<i>: every rank on device i (ranks sharing one GPU on any box -- the
        # shared-GPU tests); otherwise local rank r on device r (modulo the devices there are)
        shared = os.environ.get("PDCC_SPAWN_DEVICE", "")
        idx = int(shared) if shared else int(os.environ["LOCAL_RANK"])
        torch.cuda.set_device(idx % torch.cuda.device_count())
    kw = {}
    if timeout_s is not None:
        kw["timeout"] = datetime.timedelta(seconds=timeout_s)
    dist.init_process_group(backend, rank=rank, world_size=size, **kw)
    try:
        return fn(rank, size, *args)
    finally:
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def _child(rank, size, fn, backend, port, args, bind_device, timeout_s, q):
    try:
        res = init_process(rank, size, fn, backend, port, args, bind_device, timeout_s)
        q.put((rank, True, res))
    except BaseException as e:  # noqa: BLE001 - report everything to the parent
        q.put((rank, False, f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))
        raise SystemExit(1)


def launch(
    fn: Callable[..., Any],
    world_size: int,
    args: Sequence[Any] = (),
    backend: str = BACKEND_NAME,
    bind_device: bool = False,
    timeout_s: float | None = None,
    join_timeout_s: float = 300.0,
    env: dict | None = None,
) -> list:
    """Run ``fn(rank, world_size, *args)`` on ``world_size`` spawned processes and
    return the per-rank results (rank order). Raises if any rank fails."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    old = {}
    if env:
        for k, v in env.items():
            old[k] = os.environ.get(k)
            os.environ[k] = str(v)
    try:
        procs = [
            ctx.Process(target=_child, args=(r, world_size, fn, backend, port, args, bind_device, timeout_s, q))
            for r in range(world_size)
        ]
        for p in procs:
            p.start()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    results: dict[int, Any] = {}
    errors: dict[int, str] = {}
    import queue
    import time

    deadline = time.time() + join_timeout_s
    while len(results) + len(errors) < world_size:
        try:
            rank, ok, payload = q.get(timeout=0.2)
            (results if ok else errors)[rank] = payload
            if not ok:
                break
        except queue.Empty:
            dead = [p for p in procs if p.exitcode not in (None, 0)]
            if dead and len(results) + len(errors) < world_size:
                # give the queue a moment to deliver the error report
                time.sleep(0.5)
                while not q.empty():
                    rank, ok, payload = q.get()
                    (results if ok else errors)[rank] = payload
                if len(results) + len(errors) < world_size:
                    for p in procs:
                        if p.exitcode not in (None, 0) and procs.index(p) not in errors:
                            errors[procs.index(p)] = f"exited with code {p.exitcode}"
                break
            if time.time() > deadline:
                errors[-1] = f"timed out after {join_timeout_s}s"
                break
    if errors:
        for p in procs:
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(timeout=10)
        for p in procs:  # a rank that ignores SIGTERM (stuck in a GPU wait, or a profiler's handler
            if p.is_alive():  # chained in front of it) would block interpreter exit in its join
                p.kill()
                p.join(timeout=10)
        msg = "\n".join(f"rank {r}: {e}" for r, e in sorted(errors.items()))
        raise RuntimeError(f"distributed run failed:\n{msg}")
    for p in procs:
        p.join(timeout=30)
    bad = [(i, p.exitcode) for i, p in enumerate(procs) if p.exitcode not in (0, None)]
    if bad:
        raise RuntimeError(f"ranks exited with non-zero codes: {bad}")
    return [results[r] for r in range(world_size)]
