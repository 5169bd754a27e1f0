"""RCCL buffer / protocol sweep in fresh processes (verdict r3 Next #6).

RCCL reads ``NCCL_BUFFSIZE``, ``NCCL_PROTO`` and its other ``NCCL_*`` parameters
once per process, when the first communicator comes up. The in-process autotuner
(csrc/backend/autotune.cpp) can therefore race engines and channel counts, but
never these. This module measures them the only way they can be measured: every
candidate setting runs in a FRESH set of child ranks, one per GPU. The children
time the reference's headline collective (``dist.all_reduce`` SUM, main.py:23)
at BASELINE.json's size on this library's RCCL engine (``PDCC_ALGO=rccl``), and
rank 0's child reports the p50 over ranks (nccl-tests busbw convention).

Two drivers share one child:

* :func:`sweep` -- called by EVERY rank of a running job (``bench.py`` under
  torchrun or its own launcher) BEFORE that rank touches the GPU. Each rank
  starts its own child per point. The children rendezvous on a port that rank 0
  publishes in the job's store, and the winner is published back so every rank
  applies the same environment to its own (later) RCCL communicators.
* ``python -m pytorch_distributed_collective_communication_amd.utils.rccl_env
  --gpus N`` -- a standalone sweep that starts all N children itself and prints
  the recommended ``PDCC_RCCL_BUFFSIZE`` / ``PDCC_RCCL_PROTO`` settings (the
  backend forwards those to ``NCCL_*`` at its first communicator,
  csrc/device/rccl_comm.cpp ``forward_rccl_env``).

Points (run in this order inside a wall-clock budget; a point that would start after the
budget is recorded as skipped): RCCL's defaults; the algorithm forced to ``NCCL_ALGO=Ring``
and ``Tree``; RCCL's MSCCL all-pairs algorithms (``RCCL_MSCCL_ENABLE``, the shipped
``allreduce-allpairs-8n-*.xml``) forced on and off; ``NCCL_PROTO=Simple``; ``NCCL_BUFFSIZE``
of 16 / 32 MiB, and 16 MiB with Simple.

The verdict is persisted (:func:`persist`) keyed by a topology signature -- host, world
size, GPUs visible, RCCL version -- in ``PDCC_RCCL_ENV_FILE`` (default: next to
``PDCC_AUTOTUNE_FILE`` if that is set, else ``~/.cache/pdcc/rccl_env.json``), and every
process of this library applies it (:func:`apply_persisted`, from the backend's creator)
before its first RCCL communicator -- not only ``bench.py``. Settings the user made
(``NCCL_*`` / ``PDCC_RCCL_*``) always win.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import shutil
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import time

MiB = 1 << 20
# NCCL / RCCL variable -> the PDCC_RCCL_* name the backend forwards (csrc/device/rccl_comm.cpp)
_PDCC_NAME = {"NCCL_BUFFSIZE": "PDCC_RCCL_BUFFSIZE", "NCCL_PROTO": "PDCC_RCCL_PROTO",
              "NCCL_ALGO": "PDCC_RCCL_ALGO", "RCCL_MSCCL_ENABLE": "PDCC_RCCL_MSCCL"}
_ENV_KEYS = tuple(_PDCC_NAME)
# (name, setting): one dimension at a time from RCCL's defaults (ALGO and MSCCL are the all-pairs /
# tree alternatives SURVEY.md §5.8 asks for), then the buffer sizes that won before
_GRID = (
    ("default", {}),
    ("algo=Ring", {"NCCL_ALGO": "Ring"}),
    ("algo=Tree", {"NCCL_ALGO": "Tree"}),
    ("msccl=1", {"RCCL_MSCCL_ENABLE": "1"}),
    ("msccl=0", {"RCCL_MSCCL_ENABLE": "0"}),
    ("proto=Simple", {"NCCL_PROTO": "Simple"}),
    ("buffsize=16MiB", {"NCCL_BUFFSIZE": str(16 * MiB)}),
    ("buffsize=32MiB", {"NCCL_BUFFSIZE": str(32 * MiB)}),
    ("buffsize=16MiB,proto=Simple", {"NCCL_BUFFSIZE": str(16 * MiB), "NCCL_PROTO": "Simple"}),
)
# torchrun's agent-store variables must not leak into the children: they rendezvous among
# themselves on their own port, not through the parent job's agent
_STRIP = ("TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
          "TORCHELASTIC_MAX_RESTARTS", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME",
          "GROUP_WORLD_SIZE", "LOCAL_WORLD_SIZE", "TORCHELASTIC_ERROR_FILE")


def points():
    """The sweep grid, in run order: (name, {variable: value or None = unset})."""
    return [(name, {k: over.get(k) for k in _ENV_KEYS}) for name, over in _GRID]


def user_set() -> list:
    """RCCL settings the user made (their own NCCL_* or this library's PDCC_RCCL_* names)."""
    return [k for k in _ENV_KEYS + tuple(_PDCC_NAME.values()) if os.environ.get(k)]


def env_file() -> str | None:
    """Where sweep verdicts persist (None: PDCC_RCCL_ENV_FILE=0 / off)."""
    f = os.environ.get("PDCC_RCCL_ENV_FILE")
    if f is not None:
        return None if f.strip().lower() in ("", "0", "off", "none") else f
    tune = os.environ.get("PDCC_AUTOTUNE_FILE")
    if tune:
        return tune + ".rccl_env.json"
    return os.path.join(os.path.expanduser("~"), ".cache", "pdcc", "rccl_env.json")


def signature(world: int, ngpu: int | None = None) -> str:
    """Topology key of a verdict: host, world size, GPUs visible, RCCL version (no GPU init)."""
    try:
        import torch

        if ngpu is None:
            ngpu = torch.cuda.device_count()
        ver = torch.cuda.nccl.version()
        ver = ".".join(str(v) for v in ver) if isinstance(ver, tuple) else str(ver)
    except Exception:
        ver = "?"
    return f"{socket.gethostname()}|w{world}|g{ngpu or 0}|rccl{ver}"


def _load(path):
    try:
        with open(path) as f:
            d = json.load(f)
        return d if isinstance(d, dict) else {}
    except (OSError, ValueError):
        return {}


def persist(sig: str, rec: dict, path: str | None = None) -> str | None:
    """Record a sweep's verdict for `sig` (atomic replace; the applied env may be empty: RCCL's
    defaults won). Returns the file written, or None."""
    path = path or env_file()
    if not path:
        return None
    d = _load(path)
    d[sig] = {"env": rec.get("applied_env") or {}, "winner": rec.get("winner"), "bytes": rec.get("bytes"),
              "p50_ms": {k: v.get("p50_ms") for k, v in rec.get("points", {}).items() if isinstance(v, dict)},
              "time": time.strftime("%Y-%m-%dT%H:%M:%S")}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    os.replace(tmp, path)
    return path


applied: dict = {}  # what apply_persisted set in this process (introspection)
_checked = False


def apply_persisted(world: int, ngpu: int | None = None, path: str | None = None) -> dict:
    """Apply the persisted verdict for this topology to this process's environment, as the
    PDCC_RCCL_* names the backend forwards at its first RCCL communicator. No-op if the user set
    any RCCL variable, if no verdict matches, or once a verdict was applied. Returns what was set."""
    global applied, _checked
    if _checked or world < 2 and not os.environ.get("PDCC_RCCL_ENV_ANY_WORLD"):
        return applied
    _checked = True  # (RCCL reads its environment once per process: the first group decides)
    path = path or env_file()
    if not path or user_set():
        return {}
    ent = _load(path).get(signature(world, ngpu))
    if not ent or not isinstance(ent.get("env"), dict):
        return {}
    out = {}
    for k, v in ent["env"].items():
        if k in _PDCC_NAME and v:
            os.environ[_PDCC_NAME[k]] = str(v)
            out[_PDCC_NAME[k]] = str(v)
    applied = out
    return out


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def _child_env(rank: int, world: int, local_rank: int, port: int, over: dict, nbytes: int, iters: int,
               result: str | None):
    env = {k: v for k, v in os.environ.items() if k not in _STRIP}
    for k in _ENV_KEYS:  # the point's setting, not whatever the parent job carries
        env.pop(k, None)
        env.pop(_PDCC_NAME[k], None)
    env["PDCC_RCCL_ENV_FILE"] = "0"  # (a child never applies an earlier verdict)
    for k, v in over.items():
        if v is not None:
            env[k] = v
    env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(local_rank), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), PDCC_ALGO="rccl", PDCC_IPC="0", PDCC_AUTOTUNE="0",
               PDCC_RCCL_ENV_CHILD_BYTES=str(nbytes), PDCC_RCCL_ENV_CHILD_ITERS=str(iters))
    env.pop("PDCC_RCCL_ENV_CHILD_RESULT", None)
    if result:
        env["PDCC_RCCL_ENV_CHILD_RESULT"] = result
    return env


def _spawn(env):
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return subprocess.Popen([sys.executable, "-m", "pytorch_distributed_collective_communication_amd.utils.rccl_env",
                             "--child"], env=env, cwd=root, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            text=True, start_new_session=True)


def _reap(procs, deadline: float):
    """Wait for the children until `deadline`; kill the process groups of the late ones.
    Returns (exit codes, stderr tails)."""
    codes, tails = [], []
    for p in procs:
        try:
            _, err = p.communicate(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            _, err = p.communicate()
        codes.append(p.returncode)
        tails.append((err or "")[-400:])
    return codes, tails


def _read_result(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _decide(results: dict, min_gain: float = 0.05):
    """Winner = lowest p50 among points that ran correctly; applied only if it beats RCCL's
    defaults by `min_gain` (run-to-run noise of one short point is a few percent)."""
    ok = {k: v for k, v in results.items() if isinstance(v, dict) and v.get("ok")}
    if not ok:
        return None, None
    best = min(ok, key=lambda k: ok[k]["p50_ms"])
    base = ok.get(points()[0][0])
    apply = base is not None and ok[best]["p50_ms"] < (1.0 - min_gain) * base["p50_ms"]
    env = dict(points_env()[best]) if apply else None
    return best, env


def points_env():
    return {n: {k: v for k, v in e.items() if v is not None} for n, e in points()}


def sweep(store, rank: int, world: int, local_rank: int, nbytes: int = 1 << 30, budget_s: float = 90.0,
          point_timeout_s: float = 45.0, iters: int = 5, tag: str = "bench"):
    """Collective over the job's ranks (each calls it before its first GPU call). Returns
    the record (identical on every rank) and the environment every rank should apply."""
    t_start = time.time()
    key = f"pdcc_rccl_env/{tag}"
    results: dict = {}
    tmp = tempfile.mkdtemp(prefix="pdcc_rccl_env_") if rank == 0 else None
    wait = datetime.timedelta(seconds=point_timeout_s + 30)
    for k, (name, over) in enumerate(points()):
        if rank == 0:
            go = time.time() - t_start + point_timeout_s / 3 < budget_s
            store.set(f"{key}/go/{k}", "1" if go else "0")
            if go:
                store.set(f"{key}/port/{k}", str(free_port()))
        store.wait([f"{key}/go/{k}"], wait)
        if store.get(f"{key}/go/{k}") != b"1":
            results[name] = "skipped: sweep budget spent"
            continue
        port = int(store.get(f"{key}/port/{k}"))
        out = os.path.join(tmp, f"p{k}.json") if rank == 0 else None
        t0 = time.time()
        p = _spawn(_child_env(rank, world, local_rank, port, over, nbytes, iters, out))
        codes, tails = _reap([p], t0 + point_timeout_s)
        store.set(f"{key}/rc/{k}/{rank}", str(codes[0]))
        if rank == 0:
            rcs = []
            for r in range(world):
                try:
                    store.wait([f"{key}/rc/{k}/{r}"], wait)
                    rcs.append(int(store.get(f"{key}/rc/{k}/{r}")))
                except Exception:
                    rcs.append(None)
            rec = _read_result(out) or {}
            rec.update(ok=all(c == 0 for c in rcs) and "p50_ms" in rec, rc=rcs, wall_s=round(time.time() - t0, 2))
            if not rec["ok"]:
                rec["stderr_tail"] = tails[0]
            results[name] = rec
    out_rec = None
    if rank == 0:
        best, env = _decide(results)
        out_rec = {"points": results, "winner": best, "applied_env": env, "min_gain": 0.05,
                   "bytes": nbytes, "iters": iters, "elapsed_s": round(time.time() - t_start, 1)}
        if best is not None:  # (only a sweep that measured something is a verdict)
            try:
                out_rec["persisted"] = {"file": persist(signature(world), out_rec), "signature": signature(world)}
            except OSError as e:
                out_rec["persisted"] = {"error": str(e)[:200]}
        store.set(f"{key}/record", json.dumps(out_rec))
        shutil.rmtree(tmp, ignore_errors=True)
    store.wait([f"{key}/record"], wait)
    out_rec = json.loads(store.get(f"{key}/record"))
    return out_rec, out_rec.get("applied_env") or {}


def sweep_local(world: int, nbytes: int = 1 << 30, budget_s: float = 300.0, point_timeout_s: float = 60.0,
                iters: int = 5):
    """Standalone sweep: this process starts all `world` children of every point itself."""
    t_start = time.time()
    results = {}
    tmp = tempfile.mkdtemp(prefix="pdcc_rccl_env_")
    for k, (name, over) in enumerate(points()):
        if time.time() - t_start + point_timeout_s / 3 >= budget_s:
            results[name] = "skipped: sweep budget spent"
            continue
        port, out, t0 = free_port(), os.path.join(tmp, f"p{k}.json"), time.time()
        procs = [_spawn(_child_env(r, world, r, port, over, nbytes, iters, out if r == 0 else None))
                 for r in range(world)]
        codes, tails = _reap(procs, t0 + point_timeout_s)
        rec = _read_result(out) or {}
        rec.update(ok=all(c == 0 for c in codes) and "p50_ms" in rec, rc=codes, wall_s=round(time.time() - t0, 2))
        if not rec["ok"]:
            rec["stderr_tail"] = next((t for t in tails if t), "")
        results[name] = rec
    best, env = _decide(results)
    shutil.rmtree(tmp, ignore_errors=True)
    rec = {"points": results, "winner": best, "applied_env": env, "bytes": nbytes, "iters": iters,
           "elapsed_s": round(time.time() - t_start, 1)}
    if best is not None:
        rec["persisted"] = {"file": persist(signature(world), rec), "signature": signature(world)}
    return rec


def _child():
    """One rank of one sweep point: 1 GiB fp32 all_reduce on the library's RCCL engine."""
    import torch
    import torch.distributed as dist

    import pytorch_distributed_collective_communication_amd as pdcc
    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    pdcc._load_native()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local % torch.cuda.device_count())
    t0 = time.perf_counter()
    dist.init_process_group("mi355x", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    n = int(os.environ["PDCC_RCCL_ENV_CHILD_BYTES"]) // 4
    iters = int(os.environ["PDCC_RCCL_ENV_CHILD_ITERS"])
    x = torch.rand(n, device="cuda").mul_(1e-3)
    dist.all_reduce(x)  # communicator creation
    torch.cuda.synchronize()
    init_ms = (time.perf_counter() - t0) * 1e3
    dist.all_reduce(x)
    lat = []
    for _ in range(iters):
        dist.barrier()
        torch.cuda.synchronize()
        s = time.perf_counter()
        dist.all_reduce(x)
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - s], dtype=torch.float64)
        engine = be.native_backend(None, "cuda").last_algo()  # (before the host-transport MAX below)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # CPU tensor: host transport
        lat.append(t.item())
    p50 = statistics.median(lat)
    out = os.environ.get("PDCC_RCCL_ENV_CHILD_RESULT")
    if out and rank == 0:
        from pytorch_distributed_collective_communication_amd.utils import busbw

        rec = {"p50_ms": round(p50 * 1e3, 3), "busbw_GBps": round(busbw("all_reduce", n * 4, world, p50), 1),
               "engine": engine, "init_ms": round(init_ms, 1),
               "env": {k: os.environ.get(k) for k in _ENV_KEYS if os.environ.get(k)}}
        with open(out + ".tmp", "w") as f:
            json.dump(rec, f)
        os.replace(out + ".tmp", out)
    dist.destroy_process_group()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--budget-s", type=float, default=300.0)
    a = ap.parse_args(argv)
    if a.child:
        _child()
        return
    rec = sweep_local(a.gpus, a.bytes, a.budget_s, iters=a.iters)
    print(json.dumps(rec, indent=1))
    if rec["applied_env"]:
        print("# recommended:", " ".join(f"PDCC_RCCL_{k[5:]}={v}" for k, v in rec["applied_env"].items()))
    else:
        print("# RCCL's defaults are within 5% of the best point: nothing to set")


if __name__ == "__main__":
    main()
