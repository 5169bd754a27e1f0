#!/usr/bin/env python3
"""Headline benchmark: all_reduce busbw + p50 latency, 1 GiB fp32 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]            # starts N ranks itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N  # or under torchrun

Without a torchrun environment (no WORLD_SIZE) and N > 1 the script is its own
launcher (``launch_ranks``): it starts N child ranks on a free 127.0.0.1 port,
makes no GPU call itself, and propagates the first failing rank's exit code.
``PDCC_BENCH_DEVICE=cpu`` runs the same harness on CPU tensors through the
backend's host transport (functional rehearsal, used by the CPU test suite).

One rank per GPU, backend ``mi355x`` (this library). A "step" is one in-place
``dist.all_reduce(SUM)`` of a 1 GiB fp32 tensor (268,435,456 synthetic random
elements per rank). W untimed warm-up steps, then exactly K steps bracketed by
``barrier + torch.cuda.synchronize()`` on both sides; the time is the MAX over
ranks. busbw uses the nccl-tests convention ``S * 2(n-1)/n / t`` (0 at n=1,
where all_reduce is a no-op). p50 = median over K individually-bracketed steps
of the max-over-ranks time (BASELINE.md method). Rank 0 prints ONE JSON line.

Extra fields (not part of the headline): K1 kernel bandwidth on this GPU, and
for N>1 an A/B of the algorithms (RCCL vs the IPC peer-memory kernels) at the
headline size and at small sizes, each with a correctness check.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_BUSBW = {2: 6.14, 4: 5.49, 8: 3.16}  # BASELINE.md §2.1 (reference stack, Gloo/CPU)
BASELINE_P50_MS = {1: 0.027, 2: 174.8, 4: 293.4, 8: 595.1}  # same table, p50 latency
SMALL = os.environ.get("PDCC_BENCH_SMALL", "0") == "1"  # functional rehearsal sizes for the extras
# PDCC_BENCH_RCCL_REHEARSAL=1 (world 1, one GPU): run the RCCL-only extras the driver's multi-GPU
# node would run first -- the RCCL environment pre-sweep in fresh child ranks, torch's own
# ProcessGroupNCCL comparator, the RCCL A/B, the baseline rows, the CTA sweep / list all-gather /
# group churn -- on 1-rank communicators (PDCC_WORLD1_LOCAL=0: the library's RCCL engine runs even
# where all_reduce is a no-op), so none of them first executes on the scaling run
REHEARSAL = os.environ.get("PDCC_BENCH_RCCL_REHEARSAL", "0") == "1"
NBYTES = 1 << 30
EXTRAS_PARTIAL: dict = {}  # run_extras fills this in place (reported even if a deadline fires)
# wall seconds per section of this rank's run (extras.timing; rank 0's view): on the first
# multi-GPU node every first call pays for communicators, self-tests and autotune races
TIMING: dict = {}
EXTRAS_PARTIAL["timing"] = TIMING
T_START = time.time()


class section:
    """``with section("name"):`` adds the block's wall seconds to extras.timing[name]."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.t0 = time.time()
        return self

    def __exit__(self, *exc):
        TIMING[self.name] = round(TIMING.get(self.name, 0.0) + time.time() - self.t0, 3)
        return False


def busbw(nbytes: int, n: int, sec: float) -> float:
    return 0.0 if n <= 1 or sec <= 0 else nbytes * 2 * (n - 1) / n / sec / 1e9


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bytes", type=int, default=NBYTES)
    ap.add_argument("--extras", type=int, default=int(os.environ.get("PDCC_BENCH_EXTRAS", "1")))
    return ap.parse_args(argv)


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """``python bench.py --gpus N`` without a torchrun environment: start N
    ranks of this script as child processes (one per GPU, LOCAL_RANK = rank),
    the way the reference's ``__main__`` starts its workers (main.py:98-108) but
    with exit codes checked. This parent makes no GPU call and never imports
    torch; it waits for the ranks, and if one fails or the deadline passes it
    stops the others and exits non-zero. Only rank 0 prints the JSON line (the
    children share this process's stdout)."""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    # below the driver's own 600 s limit: if the ranks hang, this parent (not the driver) stops them
    deadline = time.time() + float(os.environ.get("PDCC_BENCH_TIMEOUT_S", "540"))
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            r, c = bad[0]
            print(f"[bench] rank {r} exited with code {c}; stopping the other ranks", file=sys.stderr, flush=True)
            rc = c if c > 0 else 128 - c
            break
        if all(c == 0 for c in codes):
            break
        if time.time() > deadline:
            print("[bench] deadline passed; stopping the ranks", file=sys.stderr, flush=True)
            rc = 124
            break
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t_end = time.time() + 15
    for p in procs:
        try:
            p.wait(timeout=max(0.1, t_end - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, argv))
    run_rank(args)


def run_rank(args):
    if os.environ.get("PDCC_BENCH_DEBUG_S"):
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["PDCC_BENCH_DEBUG_S"]), exit=True)

    import torch
    import torch.distributed as dist

    import pytorch_distributed_collective_communication_amd as pdcc
    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    pdcc._load_native()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    on_gpu = os.environ.get("PDCC_BENCH_DEVICE", "cuda") != "cpu"
    if REHEARSAL:
        if world != 1 or not on_gpu:
            raise SystemExit("PDCC_BENCH_RCCL_REHEARSAL=1 is a world-1 GPU rehearsal (--gpus 1)")
        os.environ["PDCC_WORLD1_LOCAL"] = "0"  # before the pre-sweep's children and our own group
    TIMING["startup"] = round(time.time() - T_START, 3)
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
    # the job's store first (torch's own env:// rendezvous, agent store under torchrun): the
    # RCCL environment pre-sweep below runs over it before this process touches the GPU
    with section("rendezvous"):
        from torch.distributed import rendezvous

        store, _, _ = next(rendezvous("env://", rank, world, timeout=datetime.timedelta(minutes=10)))
    # counting devices does not initialise the GPU on this runtime; set_device does
    ngpu = torch.cuda.device_count() if on_gpu else 0
    with section("rccl_env_sweep"):
        EXTRAS_PARTIAL["rccl_env_sweep"] = rccl_env_presweep(store, rank, world, local, on_gpu, ngpu, args)
    if on_gpu and ngpu < world:
        # ranks sharing a GPU (functional rehearsals only): each process's streams take their own
        # hardware queues, and past the number the GPU maps at once the hardware time-slices them
        # -- a rank's IPC kernel then waits a scheduling quantum for its peer (W = 8 after the
        # conformance pass: 56 ms per op at unchanged kernel bodies, scripts/queue_slicing_probe.py,
        # profiles/r5/). GPU_MAX_HW_QUEUES=1 per rank (set before the ranks start) avoids it; the
        # record says which it was.
        q = os.environ.get("GPU_MAX_HW_QUEUES", "")
        EXTRAS_PARTIAL["shared_gpu"] = {"ranks": world, "gpus": ngpu, "gpu_max_hw_queues": q or "default",
                                        "may_time_slice": q != "1"}
    if on_gpu:
        local = local % ngpu  # (ranks > GPUs only in functional rehearsals on a 1-GPU box)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:  # functional rehearsal of the whole harness on the host transport (tests)
        dev = torch.device("cpu")
        torch.set_num_threads(1)
    csync = torch.cuda.synchronize if on_gpu else (lambda: None)
    with section("init_process_group"):
        dist.init_process_group("mi355x", store=store, rank=rank, world_size=world,
                                timeout=datetime.timedelta(minutes=10))
    native = be.native_backend()

    numel = args.bytes // 4
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.rand(numel, device=dev, generator=gen).mul_(1e-3)
    # in-place SUM multiplies the data by W per step (+inf after ~43 steps at W=8): every
    # phase starts from this copy again (restored outside the timed regions)
    x0 = x.clone()

    def sync():
        dist.barrier()
        csync()

    def max_over_ranks(v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)  # CPU tensor: host transport
        return t.item()

    # warm-up; the first call sets the GPU path up (topology, IPC self-test, communicators,
    # the autotune race for this size) and is timed on its own
    with section("first_call"):
        if args.warmup > 0:
            dist.all_reduce(x)
        csync()
    with section("warmup"):
        for _ in range(max(0, args.warmup - 1)):
            dist.all_reduce(x)
        x.copy_(x0)
        sync()
    if rank == 0:
        print(f"[bench] world={world} warm-up done, timing {args.steps} steps", file=sys.stderr, flush=True)
    zc0 = zc_counters(native)  # (zero-copy outcomes of the timed steps: deltas in the record)
    # ---- the timed region: exactly K steps
    with section("timed"):
        t0 = time.perf_counter()
        for _ in range(args.steps):
            dist.all_reduce(x)
        algo = native.last_algo() or "?"  # the engine that served the timed steps
        csync()
        dist.barrier()
        csync()
        total = max_over_ranks(time.perf_counter() - t0)
    zc_timed = zc_delta(zc0, zc_counters(native), max_over_ranks)
    finite = bool(torch.isfinite(x).all().item())
    ms_per_step = total / args.steps * 1e3

    # ---- p50 of individually bracketed steps (BASELINE.md method)
    with section("p50_steps"):
        lat = []
        for _ in range(args.steps):
            x.copy_(x0)
            sync()
            s0 = time.perf_counter()
            dist.all_reduce(x)
            csync()
            lat.append(max_over_ranks(time.perf_counter() - s0))
        p50 = statistics.median(lat)
        finite = finite and bool(torch.isfinite(x).all().item())
        x.copy_(x0)
        del x0

    # ---- correctness of the headline path
    with section("correctness"):
        y = torch.full((numel,), float(rank + 1), device=dev)
        dist.all_reduce(y)
        exp = world * (world + 1) / 2
        correct = bool(torch.all(y == exp).item())
        del y

    value = busbw(args.bytes, world, ms_per_step / 1e3)
    try:  # the autotuner's decisions for the headline path (size bucket -> engine, times)
        EXTRAS_PARTIAL["autotune"] = native.autotune_table()
    except Exception:
        pass

    def headline(extras):
        return {
            "metric": "all_reduce busbw (GB/s) + p50 latency, 1 GiB fp32",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "p50_ms": round(p50 * 1e3, 4),
            "baseline_p50_ms": BASELINE_P50_MS.get(world),
            "busbw_p50_GBps": round(busbw(args.bytes, world, p50), 3),
            "algbw_GBps": round(args.bytes / (ms_per_step / 1e3) / 1e9, 3) if world > 1 else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_BUSBW[world], 2) if world in BASELINE_BUSBW else None,
            "dtype": "fp32",
            "data": f"synthetic (torch.rand, {args.bytes} bytes fp32 per rank, random-init; no dataset)",
            "config": {
                "model": "all_reduce SUM 1 GiB fp32 (reference main.py do_all_reduce, scaled to BASELINE.json)",
                "global_batch": world,
                "seq_len": numel,
                "parallelism": f"dp{world}",
                "backend": "mi355x",
                "algo": algo,
                "device": dev.type,
                # the engine label is the outcome (verdict r5 Next #1); these say how many of the
                # timed calls attempted zero copy and fell back to staging, MAX over ranks
                "zc_timed": zc_timed,
            },
            "correct": correct,
            "data_finite": finite,
            # torch's own ProcessGroupNCCL on the same 1 GiB all_reduce (extras.torch_nccl): its p50 / ours
            "vs_torch_nccl": _vs_torch_nccl_headline(extras, p50, args.bytes),
            "note": ("world=1: all_reduce is a no-op, busbw is 0 by the nccl-tests definition"
                     + ("; RCCL rehearsal (1-rank communicators, PDCC_WORLD1_LOCAL=0)" if REHEARSAL else ""))
                    if world == 1 else "",
            "extras": extras,
        }

    # The headline is already measured: whatever the extras do (a stuck peer on a
    # new topology, say), the JSON line gets printed and the process exits.
    printed = threading.Lock()

    def emit(extras):
        if rank == 0 and printed.acquire(blocking=False):
            print(json.dumps(headline(extras)), flush=True)

    def deadline(what):
        emit({"error": f"{what} exceeded its deadline", "partial": dict(EXTRAS_PARTIAL)})
        sys.stderr.flush()
        os._exit(0)

    extras = {}
    if args.extras:
        timer = threading.Timer(float(os.environ.get("PDCC_BENCH_EXTRAS_S", "240")), deadline, args=("extras",))
        timer.daemon = True
        timer.start()
        # the conformance pass first: on the driver's multi-GPU node this is the first
        # distinct-GPU run of every engine, so its verdict must not wait behind the sweeps
        try:
            from pytorch_distributed_collective_communication_amd.utils import conformance

            progress("conformance pass")
            with section("conformance"):
                EXTRAS_PARTIAL["conformance"] = conformance.run(
                    rank, world, dev, deadline_s=float(os.environ.get("PDCC_BENCH_CONFORMANCE_S", "45")),
                    max_bytes=(64 << 20) if on_gpu and not SMALL else (1 << 20))
        except Exception as e:
            EXTRAS_PARTIAL["conformance"] = {"all_ok": False, "error": f"{type(e).__name__}: {e}"[:500]}
        if on_gpu:
            try:
                extras = run_extras(world, rank, dev, native, x)
            except Exception as e:  # extras never break the headline line
                extras = dict(EXTRAS_PARTIAL)
                extras["error"] = f"{type(e).__name__}: {e}"[:500]
        else:
            EXTRAS_PARTIAL["torch_nccl"] = {"skipped": "CPU rehearsal (PDCC_BENCH_DEVICE=cpu): no GPU"}
            extras = dict(EXTRAS_PARTIAL)
        timer.cancel()
    TIMING["total"] = round(time.time() - T_START, 3)
    emit(extras)
    guard = threading.Timer(60.0, lambda: os._exit(0))  # teardown must not hang the job either
    guard.daemon = True
    guard.start()
    dist.destroy_process_group()


def rccl_env_presweep(store, rank, world, local, on_gpu, ngpu, args):
    """RCCL reads NCCL_BUFFSIZE / NCCL_PROTO once per process: measure them in fresh child
    ranks before this rank touches the GPU (utils/rccl_env.py), and apply the winner to this
    rank's own communicators (every rank applies the same one). Distinct GPUs only."""
    if not on_gpu:
        return {"skipped": "CPU rehearsal (PDCC_BENCH_DEVICE=cpu)"}
    if world < 2 and not REHEARSAL:
        return {"skipped": "world=1: no communicator to tune"}
    if ngpu < world:
        return {"skipped": f"ranks share a GPU ({world} ranks, {ngpu} GPU): RCCL refuses duplicate devices"}
    if os.environ.get("PDCC_BENCH_RCCL_ENV_SWEEP", "1") == "0":
        return {"skipped": "PDCC_BENCH_RCCL_ENV_SWEEP=0"}
    from pytorch_distributed_collective_communication_amd.utils import rccl_env

    if rccl_env.user_set():
        return {"skipped": f"RCCL settings made by the user: {rccl_env.user_set()}"}

    if rank == 0:
        print("[bench] RCCL environment pre-sweep (fresh child ranks per point)", file=sys.stderr, flush=True)
    try:
        rec, env = rccl_env.sweep(store, rank, world, local, nbytes=min(args.bytes, 64 << 20) if SMALL else args.bytes,
                                  budget_s=float(os.environ.get("PDCC_BENCH_RCCL_ENV_SWEEP_S", "90")))
    except Exception as e:  # never in the way of the headline
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    for k, v in env.items():
        os.environ[rccl_env._PDCC_NAME[k]] = v  # before this process's first RCCL communicator
    return rec


def _time_op(fn, iters, warm=2):
    import torch
    import torch.distributed as dist

    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def run_extras(world, rank, dev, native, x):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd import ops

    out = EXTRAS_PARTIAL  # filled in place, so a deadline still reports what finished
    with section("k1"):
        run_k1(world, dev, out)
    if world == 1 and not REHEARSAL:
        out["torch_nccl"] = {"skipped": "world=1: all_reduce is a no-op"}
        return out
    if world > 1:
        out["links"] = link_summary(world)
    # torch's own ProcessGroupNCCL over the same RCCL first: the bar this library must beat
    with section("torch_nccl"):
        try:
            out["torch_nccl"] = torch_nccl_compare(world, rank, dev, native, x)
        except Exception as e:
            out["torch_nccl"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    with section("algo_ab"):
        stopped = algo_ab(world, rank, dev, native, x, out)
    if not stopped:
        with section("baseline_configs"):
            try:
                out["baseline_configs"] = baseline_configs(world, rank, dev, x)
            except Exception as e:
                out["baseline_configs_error"] = f"{type(e).__name__}: {e}"[:300]
        try:  # the autotuner's verdicts for every key the baseline rows raced (default group)
            out["autotune_after_baselines"] = native.autotune_table()
        except Exception:
            pass
        if isinstance(out.get("torch_nccl"), dict) and isinstance(out.get("baseline_configs"), dict):
            out["torch_nccl"]["vs_torch_nccl"] = vs_torch_nccl(out["baseline_configs"], out["torch_nccl"])
        with section("graph_replay"):
            out.update(graph_replay(world, rank, dev))
        with section("rccl_tuning"):
            try:
                out["rccl_tuning"] = rccl_tuning(world, rank, dev, x)
            except Exception as e:
                out["rccl_tuning_error"] = f"{type(e).__name__}: {e}"[:300]
        if world > 1:  # (the IPC engines need peers)
            with section("ipc_grid_sweep"):
                try:
                    out["ipc_grid_sweep_allreduce_busbw"] = ipc_grid_sweep(world, rank, dev, x)
                except Exception as e:
                    out["ipc_grid_sweep_error"] = f"{type(e).__name__}: {e}"[:300]
    return out


def run_k1(world, dev, out):
    """K1 on this GPU: 2-source fp32 reduce of 256 MiB per source: LDS-DMA vs register staging,
    the non-temporal LDS-DMA default and the streaming kernel, and torch.add on the same data."""
    import torch

    from pytorch_distributed_collective_communication_amd import ops

    n = 64 << 20
    a = torch.rand(n, device=dev)
    b = torch.rand(n, device=dev)
    c = torch.empty_like(a)
    for impl in ("lds", "regs", "lds_ntl", "stream_ntl"):
        t = _time_op(lambda: ops.reduce_nway([a, b], out=c, impl=impl), 10) if world > 1 else _time_local(
            lambda: ops.reduce_nway([a, b], out=c, impl=impl), 10)
        out[f"k1_2src_f32_{impl}_GBps"] = round(3 * n * 4 / t / 1e9, 1)
    t = _time_op(lambda: torch.add(a, b, out=c), 10) if world > 1 else _time_local(
        lambda: torch.add(a, b, out=c), 10)
    out["torch_add_2src_f32_GBps"] = round(3 * n * 4 / t / 1e9, 1)
    ops.reduce_nway([a, b], out=c)
    ok = bool(torch.allclose(c, a + b))
    out["k1_correct"] = ok
    del a, b, c


def algo_ab(world, rank, dev, native, x, out):
    """Each engine forced in turn on the all_reduce sizes and three other collectives; returns
    True if the ranks stopped after an engine that failed (the rest of the extras is skipped)."""
    import torch
    import torch.distributed as dist

    # algorithm A/B on a short-timeout subgroup (a stuck peer aborts in 60 s, not 10 min)
    g = dist.new_group(list(range(world)), timeout=datetime.timedelta(seconds=60))
    gb = g._get_backend(torch.device("cuda"))
    flag = torch.ones(1)

    def agree(ok_local: bool) -> bool:
        f = torch.tensor([1.0 if ok_local else 0.0])
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        return f.item() > 0

    big = min((1 << 30) if not SMALL else (64 << 20), x.numel() * 4)
    rccl_ok = "rccl_ok=1" in native.describe()
    algos = ("rccl", "ipc", "ipc_push", "ipc_dyn") if rccl_ok else ("ipc", "ipc_push", "ipc_dyn")
    if world == 1:  # RCCL rehearsal: no IPC engine at world 1
        algos = ("rccl", "rccl_wide")
    if not rccl_ok:
        out["rccl_rows"] = "dropped: ranks share a GPU, RCCL unavailable"
    for algo in algos:
        try:
            gb.set_algo(algo)
            progress(f"algo A/B: {algo}")
            for nbytes in (4, 64 << 10, 1 << 20, 16 << 20, 256 << 20, big):
                if nbytes == 256 << 20 and SMALL or (algo in ("ipc_push", "ipc_dyn") and nbytes < (1 << 20)):
                    continue
                t = x[: nbytes // 4]
                lat = _time_op(lambda: dist.all_reduce(t, group=g), 10 if nbytes >= (16 << 20) else 50)
                out[f"allreduce_{algo}_{nbytes}B_us"] = round(lat * 1e6, 1)
                out[f"allreduce_{algo}_{nbytes}B_engine"] = gb.last_algo()  # what actually ran
                if nbytes >= (1 << 20):
                    out[f"allreduce_{algo}_{nbytes}B_busbw"] = round(busbw(nbytes, world, lat), 1)
                t.uniform_(0.0, 1e-3)  # in-place SUM grew it by W per call: fresh finite data
            v = torch.full((1 << 20,), float(rank + 1), device=dev)
            dist.all_reduce(v, group=g)
            good = bool(torch.all(v == world * (world + 1) / 2).item())
            # the other collectives at 1 MiB and the big size (S = total bytes, nccl-tests factors)
            from pytorch_distributed_collective_communication_amd.utils import busbw as bb

            for nbytes in ((1 << 20, big) if algo not in ("ipc_push", "ipc_dyn") else ()):  # push/dyn: all_reduce only
                per = nbytes // 4 // world
                src = x[:per]
                full = torch.empty(per * world, device=dev)
                rs_out = torch.empty(per, device=dev)
                cases = {
                    "broadcast": ("broadcast", nbytes, lambda: dist.broadcast(x[: nbytes // 4], src=0, group=g)),
                    "all_gather": ("all_gather", nbytes, lambda: dist.all_gather_into_tensor(full, src, group=g)),
                    "reduce_scatter": ("reduce_scatter", nbytes,
                                       lambda: dist.reduce_scatter_tensor(rs_out, x[: per * world], group=g)),
                }
                for name, (coll, total, fn) in cases.items():
                    lat = _time_op(fn, 10 if nbytes >= (16 << 20) else 30)
                    out[f"{name}_{algo}_{nbytes}B_us"] = round(lat * 1e6, 1)
                    out[f"{name}_{algo}_{nbytes}B_engine"] = gb.last_algo()
                    out[f"{name}_{algo}_{nbytes}B_busbw"] = round(bb(coll, total, world, lat), 1)
                ag_in = torch.full((per,), float(rank), device=dev)
                dist.all_gather_into_tensor(full, ag_in, group=g)
                good = good and bool(torch.equal(full.view(world, per)[:, 0].cpu(),
                                                  torch.arange(world, dtype=torch.float32)))
                del full, ag_in, rs_out
            out[f"allreduce_{algo}_correct"] = good
        except Exception as e:
            out[f"allreduce_{algo}_error"] = f"{type(e).__name__}: {e}"[:300]
            good = False
        if not agree(good):
            out["stopped_after"] = algo
            break
    try:
        gb.set_algo("auto")
    except Exception:
        pass
    return "stopped_after" in out


def link_summary(world):
    """How the ranks' GPUs (cuda:0..world-1, one per rank) are connected, as the HIP
    runtime reports it: counts of (link type, hops) over the ordered pairs, e.g.
    {"xgmi/1": 56} for a fully connected 8-GPU xGMI node."""
    import pytorch_distributed_collective_communication_amd as pdcc

    counts: dict = {}
    try:
        for e in pdcc._load_native().device_links():
            if e["src"] < world and e["dst"] < world:
                k = f"{e['link']}/{e.get('hops', '?')}" + ("" if e.get("p2p", 1) else "/no_p2p")
                counts[k] = counts.get(k, 0) + 1
    except Exception as e:  # informational only
        return {"error": f"{type(e).__name__}: {e}"[:200]}
    return counts


def _group_with_env(world, env, timeout_s=60):
    """A new full group whose backend reads `env` at construction (PDCC_* knobs are
    per group), built with a fresh RCCL communicator so per-communicator settings
    (channel bounds) take effect."""
    import torch.distributed as dist

    saved = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return dist.new_group(list(range(world)), timeout=datetime.timedelta(seconds=timeout_s))
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def rccl_tuning(world, rank, dev, x):
    """RCCL on this node's xGMI (only where ranks sit on distinct GPUs):
    * cta_sweep: 1 GiB all_reduce busbw at RCCL's default and at exactly 28/56/112 channels
      (minCTAs = maxCTAs) -- one CTA drives one channel, and a GPU has 7 xGMI links to saturate (the autotuner
      races the 112-channel child communicator, PDCC_RCCL_WIDE_CTAS, for large keys);
    * list_all_gather: all_gather into separate tensors, grouped p2p straight into the
      list (zero copy) vs ring all_gather into staging + K2 unpack;
    * group_churn: new_group(range(n)) + first all_reduce, as every reference demo does."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be
    from pytorch_distributed_collective_communication_amd.utils import busbw as bb

    if "rccl_ok=1" not in be.native_backend(None, "cuda").describe():
        return {"skipped": "ranks share a GPU: RCCL unavailable"}
    res = {}
    big = x if not SMALL else x[: (64 << 20) // 4]
    sweep = {}
    for ctas in ("default", 28, 56, 112):
        progress(f"rccl cta sweep: {ctas}")
        env = {"PDCC_RCCL_GROUP_COMM": "init", "PDCC_ALGO": "rccl"}
        if ctas != "default":
            env["PDCC_RCCL_MIN_CTAS"] = env["PDCC_RCCL_MAX_CTAS"] = ctas  # exact counts
        g = _group_with_env(world, env)
        t = _p50_coll(lambda: dist.all_reduce(big, group=g), iters=5)
        sweep[str(ctas)] = round(bb("all_reduce", big.numel() * 4, world, t), 1)
        big.uniform_(0.0, 1e-3)  # in-place SUM grew it by W per call: fresh finite data
        dist.destroy_process_group(g)
    res["cta_sweep_allreduce_busbw"] = sweep
    per = ((256 << 20) if not SMALL else (16 << 20)) // 4
    src = torch.full((per,), float(rank), device=dev)
    for mode in ("p2p", "staged"):
        progress(f"list all_gather: {mode}")
        g = _group_with_env(world, {"PDCC_LIST_GATHER": mode, "PDCC_ALGO": "rccl"})
        outs = [torch.empty(per + 64, device=dev)[:per] for _ in range(world)]  # never adjacent
        t = _p50_coll(lambda: dist.all_gather(outs, src, group=g), iters=5)
        ok = all(bool(outs[r][0].item() == r and outs[r][-1].item() == r) for r in range(world))
        res[f"list_all_gather_{mode}"] = {"per_rank_bytes": per * 4, "p50_ms": round(t * 1e3, 3),
                                          "busbw_GBps": round(bb("all_gather", per * 4 * world, world, t), 1),
                                          "correct": ok}
        del outs
        dist.destroy_process_group(g)
    churn = []
    for _ in range(3):
        dist.barrier()
        t0 = time.perf_counter()
        g = dist.new_group(list(range(world)))
        y = torch.ones(1024, device=dev)
        dist.all_reduce(y, group=g)
        torch.cuda.synchronize()
        churn.append(round((time.perf_counter() - t0) * 1e3, 2))
    res["group_churn_ms"] = churn
    return res


def ipc_grid_sweep(world, rank, dev, x):
    """1 GiB all_reduce busbw of the IPC pull (ipc) and push protocols for workgroup caps
    256/512/1024 (PDCC_IPC_GRID): more workgroups = more remote reads / writes in flight
    per xGMI link. (Ranks sharing a GPU are capped at 256 / W whatever the knob says.)"""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.utils import busbw as bb

    big = x if not SMALL else x[: (64 << 20) // 4]
    gsweep = {}
    for algo in ("ipc", "ipc_push"):
        for grid in (256, 512, 1024):
            progress(f"ipc grid sweep: {algo} {grid}")
            g = _group_with_env(world, {"PDCC_ALGO": algo, "PDCC_IPC_GRID": grid})
            t = _p50_coll(lambda: dist.all_reduce(big, group=g), iters=5)
            gsweep[f"{algo}_g{grid}"] = round(bb("all_reduce", big.numel() * 4, world, t), 1)
            big.uniform_(0.0, 1e-3)
            dist.destroy_process_group(g)
    v = torch.full((1 << 22,), float(rank + 1), device=dev)
    g = _group_with_env(world, {"PDCC_ALGO": "ipc", "PDCC_IPC_GRID": 1024})
    dist.all_reduce(v, group=g)
    gsweep["correct_g1024"] = bool(torch.all(v == world * (world + 1) / 2).item())
    dist.destroy_process_group(g)
    return gsweep


def graph_replay(world, rank, dev, n_ops=16, numel=1024):
    """hipGraph replay vs eager issue of a launch-bound step: n_ops small
    all_reduces captured with parallel.graphs.capture, checked afterwards.
    (With ranks sharing one GPU -- rehearsals only -- the processes' hardware
    queues get time-sliced after the capture and replays look slow; see
    scripts/graph_bench.py. One process per GPU is not affected.)"""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel.graphs import capture

    res = {}
    tag = f"graph_{n_ops}x{numel * 4}B_allreduce"
    try:
        progress("graph replay vs eager")
        bufs = [torch.zeros(numel, device=dev) for _ in range(n_ops)]

        def step():
            for b in bufs:
                dist.all_reduce(b)

        res[f"{tag}_eager_us"] = round(_time_op(step, 20) * 1e6, 1)
        g = capture(step, warmup=2)
        res[f"{tag}_replay_us"] = round(_time_op(g.replay, 20) * 1e6, 1)
        for b in bufs:
            b.fill_(float(rank + 1))
        g.replay()
        torch.cuda.synchronize()
        res[f"{tag}_correct"] = all(bool(torch.all(b == world * (world + 1) / 2).item()) for b in bufs)
    except Exception as e:
        res["graph_error"] = f"{type(e).__name__}: {e}"[:300]
    return res


def progress(msg):
    # stderr heartbeat (rank 0): long multi-GPU runs must not look hung
    import torch.distributed as dist

    if dist.get_rank() == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def zc_counters(native) -> dict:
    """The group's zero-copy outcome counters (empty on a CPU rehearsal)."""
    try:
        return dict(native.zc_counters())
    except Exception:
        return {}


def zc_delta(before: dict, after: dict, max_over_ranks=None) -> dict:
    """Per-call deltas of the counters that matter for a record (MAX over ranks if given)."""
    out = {}
    for k in ("zc_calls", "zc_fallbacks", "zc_size_refusals", "zc_full_refusals"):
        if k in after:
            v = float(after[k] - before.get(k, 0))
            out[k] = int(max_over_ranks(v) if max_over_ranks else v)
    return out


def _p50_coll(fn, iters=5):
    """BASELINE.md method: barrier + timed collective, max over ranks, median."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    fn()
    lat = []
    _p50_coll.engine = "?"
    for _ in range(iters):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        try:  # the engine that ran fn (read before the CPU-tensor MAX below records "shm")
            _p50_coll.engine = be.native_backend(_p50_coll.group, "cuda").last_algo()
        except Exception:
            pass
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lat.append(t.item())
    return statistics.median(lat)


_p50_coll.group = None  # the group whose engine _p50_coll reports (None: default group)


def baseline_configs(world, rank, dev, x, group=None, engine=None):
    """The other BASELINE.json configs on this node (default algorithm selection):
    six collectives at S = 1 GiB fp32, PRODUCT/MAX/MIN all_reduce at 128 MiB,
    all_gather bf16 4 GiB/rank (ZeRO-style), all_reduce 256 MiB at w=2.
    `group` / `engine`: the same rows on another group (torch's ProcessGroupNCCL)."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.utils import busbw as bb

    res = {}
    g = group
    _p50_coll.group = group if engine is None else None

    ours = None
    if engine is None:
        from pytorch_distributed_collective_communication_amd.parallel import backend as be

        try:
            ours = be.native_backend(group, "cuda")
        except Exception:
            ours = None

    def rec(name, coll, total_bytes, fn, iters=5, check=None):
        progress(name if engine is None else f"{engine}: {name}")
        z0 = zc_counters(ours) if ours is not None else {}
        t = _p50_coll(fn, iters)
        res[name] = {"p50_ms": round(t * 1e3, 3), "busbw_GBps": round(bb(coll, total_bytes, world, t), 1),
                     "bytes": total_bytes, "engine": engine or _p50_coll.engine}
        if ours is not None:  # this rank's zero-copy outcomes over the row's calls (warm-up + timed)
            res[name]["zc"] = zc_delta(z0, zc_counters(ours))
        if check is not None:
            res[name]["correct"] = bool(check())

    try:
        # row names carry the size actually timed (SMALL rehearsals: 64 MiB, not 1 GiB)
        S = min(1 << 30 if not SMALL else 64 << 20, x.numel() * 4)
        L = size_label(S)
        n = S // 4
        chunk = n // world
        xs = x[:n]
        xs.uniform_(0.0, 1e-3)
        tri = world * (world + 1) / 2  # sum of the fills rank + 1

        def check_all_reduce(t):  # verdict r5 Next #2: a known fill through the same call shape
            t.fill_(rank + 1.0)
            dist.all_reduce(t, group=g)
            return bool(torch.all(t == tri).item())

        def check_reduce(t):  # root: the sum; every other rank's buffer untouched
            t.fill_(rank + 1.0)
            dist.reduce(t, dst=0, group=g)
            return bool(torch.all(t == (tri if rank == 0 else rank + 1.0)).item())

        def check_broadcast(t):
            t.fill_(7.0 if rank == 0 else -1.0)
            dist.broadcast(t, src=0, group=g)
            return bool(torch.all(t == 7.0).item())

        rec(f"all_reduce_{L}", "all_reduce", S, lambda: dist.all_reduce(xs, group=g),
            check=lambda: check_all_reduce(xs))
        rec(f"reduce_{L}", "reduce", S, lambda: dist.reduce(xs, dst=0, group=g), check=lambda: check_reduce(xs))
        rec(f"broadcast_{L}", "broadcast", S, lambda: dist.broadcast(xs, src=0, group=g),
            check=lambda: check_broadcast(xs))
        src = torch.full((chunk,), float(rank), device=dev)
        out = torch.empty(n - n % world, device=dev)
        rec(f"all_gather_{L}", "all_gather", S, lambda: dist.all_gather_into_tensor(out, src, group=g),
            check=lambda: torch.equal(out.view(world, chunk)[:, 0].cpu(), torch.arange(world, dtype=torch.float32)))
        glist = [torch.empty(chunk, device=dev) for _ in range(world)] if rank == 0 else None
        rec(f"gather_{L}", "gather", S, lambda: dist.gather(src, gather_list=glist, dst=0, group=g),
            check=lambda: rank != 0 or all(bool(glist[r][0].item() == r) for r in range(world)))
        slist = [torch.full((chunk,), float(r), device=dev) for r in range(world)] if rank == 0 else None
        sout = torch.empty(chunk, device=dev)
        rec(f"scatter_{L}", "scatter", S, lambda: dist.scatter(sout, scatter_list=slist, src=0, group=g),
            check=lambda: sout[0].item() == rank)
        del glist, slist
        rsin = torch.ones(n - n % world, device=dev)
        rec(f"reduce_scatter_{L}", "reduce_scatter", S, lambda: dist.reduce_scatter_tensor(sout, rsin, group=g),
            check=lambda: sout[0].item() == world)
        a2a = torch.empty_like(rsin)
        a2a_chunk = a2a.numel() // world

        def check_a2a():  # block j of rank r goes to rank j's block r: fill r * W + j, expect j * W + r
            blocks = rsin.view(world, a2a_chunk)
            for j in range(world):
                blocks[j].fill_(float(rank * world + j))
            dist.all_to_all_single(a2a, rsin, group=g)
            want = torch.arange(world, device=dev, dtype=torch.float32) * world + rank
            return bool(torch.all(a2a.view(world, a2a_chunk) == want[:, None]).item())

        rec(f"all_to_all_{L}", "all_to_all", S, lambda: dist.all_to_all_single(a2a, rsin, group=g),
            check=check_a2a)
        del rsin, a2a, out, src
        m = ((128 << 20) if not SMALL else (8 << 20)) // 4
        pos = torch.arange(m, device=dev, dtype=torch.int64)

        def fill_op(v, op):
            # closed forms, position-dependent (a misplaced tile shows): PRODUCT of powers of two
            # (exact), MAX / MIN of small integers
            if op == "PRODUCT":
                v.copy_(torch.exp2(((pos + rank) % 3 - 1).float()))
            else:
                v.copy_(((pos % 97) * world + rank).float())

        def want_op(op):
            if op == "PRODUCT":
                e = sum(((pos + r) % 3 - 1) for r in range(world))
                return torch.exp2(e.float())
            return ((pos % 97) * world + (world - 1 if op == "MAX" else 0)).float()

        def check_op(v, op):
            fill_op(v, op)
            dist.all_reduce(v, op=getattr(dist.ReduceOp, op), group=g)
            return bool(torch.equal(v, want_op(op)))

        for op in ("PRODUCT", "MAX", "MIN"):
            v = torch.empty(m, device=dev)
            fill_op(v, op)
            rec(f"all_reduce_{op}_{size_label(m * 4)}", "all_reduce", m * 4,
                lambda: dist.all_reduce(v, op=getattr(dist.ReduceOp, op), group=g),
                check=lambda: check_op(v, op))
        del v, pos
        if world == 2:
            n2 = min(256 << 20, x.numel() * 4) // 4
            rec(f"all_reduce_{size_label(n2 * 4)}_w2", "all_reduce", n2 * 4,
                lambda: dist.all_reduce(x[:n2], group=g), check=lambda: check_all_reduce(x[:n2]))
        per = ((4 << 30) if not SMALL else (64 << 20)) // 2  # 4 GiB of bf16 per rank
        per = min(per, _shared_gpu_cap(world, dev) // 2)
        ag_in = torch.full((per,), float(rank), dtype=torch.bfloat16, device=dev)
        ag_out = torch.empty(per * world, dtype=torch.bfloat16, device=dev)
        rec(f"all_gather_bf16_{size_label(per * 2)}_per_rank", "all_gather", per * 2 * world,
            lambda: dist.all_gather_into_tensor(ag_out, ag_in, group=g), iters=3,
            check=lambda: torch.equal(ag_out.view(world, per)[:, -1].float().cpu(),
                                      torch.arange(world, dtype=torch.float32)))
        del ag_in, ag_out
    finally:
        _p50_coll.group = None
        torch.cuda.empty_cache()
    return res


def torch_nccl_compare(world, rank, dev, native, x):
    """The bar the library has to clear: torch's own ProcessGroupNCCL (``backend="nccl"``, the
    stock RCCL ProcessGroup the reference's dist.* calls would reach on GPU tensors,
    main.py:5,94) on the same tensors and the same rows as baseline_configs: the 1 GiB
    all_reduce headline, the six 1 GiB collectives, PRODUCT/MAX/MIN at 128 MiB, the bf16
    ZeRO gather. vs_torch_nccl (added by run_extras) = torch's p50 / ours per row (> 1: ours
    is faster)."""
    import torch.distributed as dist

    if "rccl_ok=1" not in native.describe():
        return {"skipped": "ranks share a GPU: RCCL (and so ProcessGroupNCCL) refuses duplicate devices"}
    progress("torch ProcessGroupNCCL comparator")
    g = dist.new_group(list(range(world)), backend="nccl", timeout=datetime.timedelta(seconds=120))
    try:
        rows = baseline_configs(world, rank, dev, x, group=g, engine="torch_nccl")
    finally:
        dist.destroy_process_group(g)
    return {"rows": rows}


def _shared_gpu_cap(world, dev) -> int:
    """Per-rank input bytes of the ZeRO-style all-gather row that fit when ranks share a GPU (rehearsals:
    W ranks x (input + W x input) on one device -- 8 x 36 GiB at full size would not fit 288 GB). The
    same value on every rank (device total, world and device count only): a power of two, at most
    40 % of the device per GPU's worth of ranks. One rank per GPU: no cap."""
    import torch

    ngpu = torch.cuda.device_count()
    if ngpu >= world:
        return 1 << 62
    per_gpu = -(-world // ngpu)
    total = torch.cuda.get_device_properties(dev).total_memory
    cap = max(1 << 20, int(0.4 * total / (per_gpu * (world + 1))))
    return 1 << (cap.bit_length() - 1)  # a power of two: the row's name stays a round size


def size_label(nbytes: int) -> str:
    """1073741824 -> '1GiB', 67108864 -> '64MiB' (row names carry the size they time)."""
    for unit, shift in (("GiB", 30), ("MiB", 20), ("KiB", 10)):
        if nbytes >= (1 << shift) and nbytes % (1 << shift) == 0:
            return f"{nbytes >> shift}{unit}"
    return f"{nbytes}B"


def _vs_torch_nccl_headline(extras, p50_s, nbytes):
    """torch's p50 / ours for the headline all_reduce, if the comparator timed that same size."""
    try:
        row = extras["torch_nccl"]["rows"][f"all_reduce_{size_label(nbytes)}"]
        return round(row["p50_ms"] / (p50_s * 1e3), 3) if p50_s > 0 else None
    except (KeyError, TypeError):
        return None


def vs_torch_nccl(ours: dict, theirs: dict) -> dict:
    rows = theirs.get("rows", {}) if isinstance(theirs, dict) else {}
    out = {}
    for k, v in rows.items():
        o = ours.get(k)
        if isinstance(o, dict) and o.get("p50_ms") and v.get("p50_ms"):
            out[k] = round(v["p50_ms"] / o["p50_ms"], 3)
    return out


def _time_local(fn, iters):
    import torch

    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


if __name__ == "__main__":
    main()
