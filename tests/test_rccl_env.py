"""The RCCL environment pre-sweep's coordination (utils/rccl_env.py) on CPU: every rank of
a job runs `sweep` over the job's store, each starts one child per point, rank 0 collects
the children's exit codes and its own child's result, decides, and every rank gets the
same record and environment back. The children are stand-ins here (no GPU): a tiny
Python process that writes the p50 the test scripts for each point."""
import json
import os
import subprocess
import sys
import threading

import pytest
import torch.distributed as dist

from pytorch_distributed_collective_communication_amd.utils import rccl_env


def _fake_spawn(p50_by_point, fail_rank=None):
    names = [n for n, _ in rccl_env.points()]

    def spawn(env):
        bs, proto = env.get("NCCL_BUFFSIZE"), env.get("NCCL_PROTO")
        name = next(n for n, e in rccl_env.points() if e["NCCL_BUFFSIZE"] == bs and e["NCCL_PROTO"] == proto)
        out = env.get("PDCC_RCCL_ENV_CHILD_RESULT")
        rc = 1 if fail_rank is not None and int(env["RANK"]) == fail_rank and name == names[1] else 0
        rec = {"p50_ms": p50_by_point[name], "busbw_GBps": 1.0, "engine": "rccl",
               "env": {k: v for k, v in (("NCCL_BUFFSIZE", bs), ("NCCL_PROTO", proto)) if v}}
        code = f"import json,sys; out={out!r}\nif out: json.dump({rec!r}, open(out, 'w'))\nsys.exit({rc})"
        assert env["PDCC_ALGO"] == "rccl" and "TORCHELASTIC_USE_AGENT_STORE" not in env
        return subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                text=True, start_new_session=True)

    return spawn


def _run(world, monkeypatch, p50, budget_s=60.0, fail_rank=None):
    monkeypatch.setattr(rccl_env, "_spawn", _fake_spawn(p50, fail_rank))
    monkeypatch.setenv("TORCHELASTIC_USE_AGENT_STORE", "True")  # must not reach the children
    store = dist.HashStore()
    out = [None] * world

    def rank(r):
        out[r] = rccl_env.sweep(store, r, world, r, nbytes=1 << 20, budget_s=budget_s, point_timeout_s=30)

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert all(o is not None for o in out)
    return out


def test_sweep_applies_a_clear_winner_on_every_rank(monkeypatch):
    names = [n for n, _ in rccl_env.points()]
    p50 = {n: 10.0 for n in names}
    p50["buffsize=16MiB,proto=Simple"] = 8.0  # 20 % better than RCCL's defaults
    out = _run(3, monkeypatch, p50)
    for rec, env in out:
        assert rec == out[0][0]
        assert rec["winner"] == "buffsize=16MiB,proto=Simple"
        assert env == {"NCCL_BUFFSIZE": str(16 << 20), "NCCL_PROTO": "Simple"}
        assert all(rec["points"][n]["ok"] for n in names)


def test_sweep_keeps_defaults_within_noise_and_drops_failed_points(monkeypatch):
    names = [n for n, _ in rccl_env.points()]
    p50 = {n: 10.0 for n in names}
    p50[names[1]] = 5.0  # fastest, but one rank's child failed there: not a candidate
    p50[names[2]] = 9.8  # within the 5 % noise band of the defaults
    out = _run(2, monkeypatch, p50, fail_rank=1)
    rec, env = out[0]
    assert rec["points"][names[1]]["ok"] is False and rec["points"][names[1]]["rc"] == [0, 1]
    assert rec["winner"] == names[2] and env == {} and rec["applied_env"] is None


def test_sweep_budget_skips_the_rest(monkeypatch):
    names = [n for n, _ in rccl_env.points()]
    out = _run(2, monkeypatch, {n: 10.0 for n in names}, budget_s=0.0)
    rec, env = out[0]
    assert all(v == "skipped: sweep budget spent" for v in rec["points"].values()), rec
    assert rec["winner"] is None and env == {}


def test_points_grid_matches_the_documented_sweep():
    pts = rccl_env.points()
    assert len(pts) == 8 and pts[0][1] == {"NCCL_BUFFSIZE": None, "NCCL_PROTO": None}
    sizes = {e["NCCL_BUFFSIZE"] for _, e in pts}
    assert sizes == {None, str(8 << 20), str(16 << 20), str(32 << 20)}
