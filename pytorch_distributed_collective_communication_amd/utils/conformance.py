"""Cross-rank conformance pass of the ``mi355x`` backend, one process per rank.

The reference verifies its six collectives by reading their printed outputs
(reference main.py:14,23,37,52,68,81; golden values README.md:105-284, SURVEY.md
§4.2). This module turns those goldens -- plus random-data numerics and the
protocol-specific paths of this library -- into a bounded pass every rank runs
together, so the first multi-GPU run of ``bench.py`` (the driver's scaling run)
is also the first distinct-GPU conformance run. Each check records whether it
passed on EVERY rank and which engine actually served it (``last_algo()``):

* ``golden/<engine>/...``  -- the reference's own calls, SUM/PRODUCT/MAX/MIN on
  ``[r+2, 10-r, r]`` for reduce / all_reduce (main.py:14-15, 23-24), scatter of
  ``[1..W]``, gather / all_gather of ``[rank]``, broadcast of ``[0]``;
* ``random/<engine>/<coll>/<dtype>/<op>/<bytes>`` -- all_reduce and
  reduce_scatter of seeded random fp32 / bf16 data against an fp64 torch
  reduction of ALL ranks' inputs (every rank regenerates them). MAX/MIN must be
  bitwise; SUM/AVG within ``(W + 1)`` units of the dtype's epsilon times
  ``sum_r |x_r|`` (engines only differ in summation order and where 16-bit
  types round); PRODUCT within ``(W + 1)`` eps of ``|prod|``;
* ``ll/<kind>`` -- all eight LL kinds (flag-tagged pushes) at 4 KiB, with the
  engine required to be ``ipc_ll`` (the list ``all_to_all`` included);
* ``zc/<...>`` -- zero-copy pull all-reduce, push all-reduce, flat all-gather,
  reduce-scatter and 2-shot broadcast at 4 MiB, engine required ``*_zc``;
* ``async_then_sync/<engine>`` -- an ``async_op=True`` all_reduce immediately
  followed by a synchronous one on the same tensor;
* ``shared_comm/<engine>`` -- two groups with the same members (one shared
  communicator) interleaving async and sync all_reduces (main.py:11,21,... build
  exactly such groups);
* ``dyn/``, ``staged/``, ``wide/``, ``rccl_wide/`` -- every other engine the
  autotuner can adopt for a key, forced: the dynamic all-gather / reduce-scatter,
  the staged (no zero copy) all-reduce / all-gather / reduce-scatter / broadcast,
  the wide-grid pull all-reduce and the wide RCCL communicator;
* ``coalesced/<engine>/...`` -- all_reduce_coalesced, all_gather_into_tensor_coalesced
  and reduce_scatter_tensor_coalesced with 64 ragged members (DDP / ZeRO buckets,
  README.md:5), on IPC and on RCCL;
* ``async_capped/<engine>/...`` -- async_op=True all_reduces on a group built with the
  opt-in PDCC_IPC_ASYNC_GRID cap (pull 2-shot and dynamic), the cap seen applied;
* ``sdma/<coll>`` -- the copy-engine engine forced for broadcast, all_gather (flat and list), gather,
  scatter and all_to_all at 4 MiB per rank, bitwise, engine required ``ipc_sdma_zc``;
* ``ops/<engine>/...`` -- PRODUCT / MAX / MIN / AVG fp32 all_reduce at 4 and 64 MiB (zero-copy and
  bulk sizes) through RCCL and every IPC engine (pull, dynamic, push, staged), plus RCCL's bulk
  reduce with every non-root buffer required bit-identical to its input;
* ``raced/...`` -- an autotuned 24 MiB fp32 SUM key whose table row must list every
  candidate as raced and valid, and an int32 BXOR key (no RCCL reduction: the IPC
  engine is the reference, checked against the host transport).

The pass stops early (every rank at the same check) once ``deadline_s`` is spent;
checks not run are listed under ``skipped``.
"""
from __future__ import annotations

import datetime
import time

_EPS = {"float32": 2.0 ** -23, "bfloat16": 2.0 ** -8, "float16": 2.0 ** -11, "float64": 2.0 ** -52}


def _seeded(shape, dtype, seed, dev, lo=-1.0, hi=1.0):
    import torch

    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.rand(shape, generator=g, device=dev, dtype=torch.float32)
    return (x * (hi - lo) + lo).to(dtype)


def _close(got, xs, op, world, dtype_name):
    """`got` (any dtype) vs the op over `xs` (list of every rank's input, same dtype)."""
    import torch

    if op in ("MAX", "MIN"):
        st = torch.stack(xs)
        ref = st.amax(0) if op == "MAX" else st.amin(0)
        return bool(torch.equal(got, ref))
    st = torch.stack([x.double() for x in xs])
    eps = _EPS[dtype_name] * (world + 1)
    g = got.double()
    if op == "PRODUCT":
        ref = st.prod(0)
        return bool(torch.all((g - ref).abs() <= eps * ref.abs() + 1e-30).item())
    ref = st.sum(0)
    bound = st.abs().sum(0)
    if op == "AVG":
        ref, bound = ref / world, bound / world
    return bool(torch.all((g - ref).abs() <= eps * bound + 1e-30).item())


class _Pass:
    def __init__(self, rank, world, dev, deadline_s):
        self.rank, self.world, self.dev = rank, world, dev
        self.t0 = time.monotonic()
        self.t_end = self.t0 + deadline_s
        self.checks: dict = {}
        self.skipped: list = []
        self.stopped = False

    def agree(self, ok: bool) -> tuple[bool, bool]:
        """(ok on every rank, every rank still inside the deadline): one host round
        on the default group, so every rank stops at the same check."""
        import torch
        import torch.distributed as dist

        v = torch.tensor([1.0 if ok else 0.0, 1.0 if time.monotonic() < self.t_end else 0.0], dtype=torch.float64)
        if self.world > 1:
            dist.all_reduce(v, op=dist.ReduceOp.MIN)
        return v[0].item() > 0, v[1].item() > 0

    def check(self, name, gb, fn, expect_engine=None):
        if self.stopped:
            self.skipped.append(name)
            return
        err = None
        # a zero-copy expectation also requires that no call of the check fell back to staging on
        # this rank (the label is the outcome of the last call; the counter covers every call)
        want_zc = expect_engine is not None and "_zc" in expect_engine
        zc0 = zc_fallbacks(gb) if want_zc else 0
        c0 = _zc_reasons(gb) if want_zc else {}
        try:
            ok = bool(fn())
        except Exception as e:  # a failing check must not stop the pass on this rank only
            ok, err = False, f"{type(e).__name__}: {e}"[:200]
        engine = gb.last_algo() if gb is not None else "?"
        if expect_engine is not None and not _engine_matches(engine, expect_engine):
            ok = False
        fb = zc_fallbacks(gb) - zc0 if want_zc else 0
        if fb:
            ok = False
        all_ok, in_time = self.agree(ok)
        rec = {"ok": all_ok, "engine": engine}
        if expect_engine is not None:
            rec["want"] = expect_engine
        if want_zc:
            rec["zc_fallbacks"] = fb
            if fb:  # why: the refusal counters that moved during the check
                c1 = _zc_reasons(gb)
                rec["zc_why"] = {k: c1[k] - c0.get(k, 0) for k in c1 if c1[k] != c0.get(k, 0)}
        if err:
            rec["error"] = err
        self.checks[name] = rec
        if not in_time:
            self.stopped = True

    def result(self):
        failed = [k for k, v in self.checks.items() if not v["ok"]]
        return {"all_ok": not failed and not self.skipped, "passed": len(self.checks) - len(failed),
                "failed": failed, "skipped": self.skipped, "elapsed_s": round(time.monotonic() - self.t0, 2),
                "checks": self.checks}


def _zc_reasons(gb) -> dict:
    """The group's zero-copy refusal counters (size guard, full mapping list, exchange fallbacks)."""
    if gb is None or not hasattr(gb, "zc_counters"):
        return {}
    c = gb.zc_counters()
    return {k: int(c.get(k, 0)) for k in ("zc_size_refusals", "zc_full_refusals", "zc_exchange_fallbacks",
                                          "zc_export_failures", "zc_map_failures")}


def zc_fallbacks(gb) -> int:
    """Calls of this group that attempted zero copy and ran staged (outcome, not intent)."""
    if gb is None or not hasattr(gb, "zc_counters"):
        return 0
    return int(gb.zc_counters().get("zc_fallbacks", 0))


def _engine_matches(engine: str, want: str) -> bool:
    if want.endswith("*"):
        return engine.startswith(want[:-1])
    return engine == want


def run(rank: int, world: int, dev, deadline_s: float = 45.0, max_bytes: int = 64 << 20,
        engines=None, timeout_s: float = 30.0) -> dict:
    """Run the pass on every rank of the default group (collective). `dev` is this
    rank's device (a GPU, or CPU for the host-transport rehearsal)."""
    import torch
    import torch.distributed as dist

    from ..parallel import backend as be

    P = _Pass(rank, world, dev, deadline_s)
    on_gpu = dev.type == "cuda"
    to = datetime.timedelta(seconds=timeout_s)
    g = dist.new_group(list(range(world)), timeout=to)
    g2 = dist.new_group(list(range(world)), timeout=to)  # same members: a shared communicator
    gb = be.native_backend(g, dev.type)
    gb2 = be.native_backend(g2, dev.type)
    # first collective sets up the group's topology (and IPC self-test) on this device
    warm = torch.zeros(1, device=dev)
    dist.all_reduce(warm, group=g)
    dist.all_reduce(warm, group=g2)
    desc = gb.describe()
    rccl_ok = "rccl_ok=1" in desc
    ipc_ok = "ipc_ok=1" in desc
    zc_ok = "zc_ok=1" in desc
    ll_ok = "ll_ok=1" in desc
    info = {"world": world, "device": dev.type, "rccl_ok": rccl_ok, "ipc_ok": ipc_ok, "zc_ok": zc_ok, "ll_ok": ll_ok,
            "zx_ok": "zx_ok=1" in desc}  # zero-copy records exchanged on the device (design.md §3)
    if engines is None:
        if not on_gpu or world == 1:
            engines = ["auto"]
        else:
            engines = (["rccl"] if rccl_ok else []) + (["ipc"] if ipc_ok else []) + ["auto"]
    if on_gpu and world > 1 and not rccl_ok:
        info["rccl_skipped"] = "ranks share a GPU: RCCL refuses duplicate devices"
    W = world
    f32 = torch.float32

    def set_engine(e):
        if hasattr(gb, "set_algo"):
            gb.set_algo(e)
            gb2.set_algo(e)

    for eng in engines:
        set_engine(eng)
        # ---- golden table, the reference's shapes
        for op in ("SUM", "PRODUCT", "MAX", "MIN"):
            rop = getattr(dist.ReduceOp, op)
            vals = [[r + 2, 10 - r, r] for r in range(W)]

            def ar(op=op, rop=rop, vals=vals):
                t = torch.tensor(vals[rank], dtype=f32, device=dev)
                dist.all_reduce(t, op=rop, group=g)
                return _close(t.cpu(), [torch.tensor(v, dtype=f32) for v in vals], op, W, "float32")

            def rd(op=op, rop=rop, vals=vals):
                t = torch.tensor(vals[rank], dtype=f32, device=dev)
                dist.reduce(t, dst=0, op=rop, group=g)
                if rank != 0:  # non-root buffers are left untouched
                    return t.cpu().tolist() == [float(v) for v in vals[rank]]
                return _close(t.cpu(), [torch.tensor(v, dtype=f32) for v in vals], op, W, "float32")

            P.check(f"golden/{eng}/all_reduce/{op}", gb, ar)
            P.check(f"golden/{eng}/reduce/{op}", gb, rd)

        def scatter():
            t = torch.empty(1, device=dev)
            lst = [torch.tensor([i + 1.0], device=dev) for i in range(W)] if rank == 0 else []
            dist.scatter(t, scatter_list=lst, src=0, group=g)
            return t.item() == rank + 1.0

        def gather():
            t = torch.tensor([float(rank)], device=dev)
            lst = [torch.empty(1, device=dev) for _ in range(W)] if rank == 0 else []
            dist.gather(t, gather_list=lst, dst=0, group=g)
            return rank != 0 or [x.item() for x in lst] == [float(r) for r in range(W)]

        def all_gather():
            lst = [torch.empty(1, device=dev) for _ in range(W)]
            dist.all_gather(lst, torch.tensor([float(rank)], device=dev), group=g)
            return [x.item() for x in lst] == [float(r) for r in range(W)]

        def broadcast():
            t = torch.tensor([0.0], device=dev) if rank == 0 else torch.full((1,), -7.0, device=dev)
            dist.broadcast(t, src=0, group=g)
            return t.item() == 0.0

        for name, fn in (("scatter", scatter), ("gather", gather), ("all_gather", all_gather),
                         ("broadcast", broadcast)):
            P.check(f"golden/{eng}/{name}", gb, fn)

        # ---- random data vs an fp64 reduction of every rank's seeded input
        sizes = [s for s in (4, 64 << 10, 1 << 20, 64 << 20) if s <= max_bytes]
        for dtn in ("float32", "bfloat16"):
            dt = getattr(torch, dtn)
            es = torch.tensor([], dtype=dt).element_size()
            for nbytes in sizes:
                n = max(1, nbytes // es)
                seed = 1000 * nbytes + (17 if dtn == "bfloat16" else 0)

                def ar_rand(n=n, dt=dt, dtn=dtn, seed=seed):
                    xs = [_seeded((n,), dt, seed + r, dev) for r in range(W)]
                    t = xs[rank].clone()
                    dist.all_reduce(t, group=g)
                    return _close(t, xs, "SUM", W, dtn)

                def rs_rand(n=n, dt=dt, dtn=dtn, seed=seed):
                    m = max(1, n // W)
                    xs = [_seeded((m * W,), dt, seed + 7 + r, dev) for r in range(W)]
                    out = torch.empty(m, dtype=dt, device=dev)
                    dist.reduce_scatter_tensor(out, xs[rank].clone(), group=g)
                    return _close(out, [x[rank * m:(rank + 1) * m] for x in xs], "SUM", W, dtn)

                P.check(f"random/{eng}/all_reduce/{dtn}/SUM/{nbytes}", gb, ar_rand)
                P.check(f"random/{eng}/reduce_scatter/{dtn}/SUM/{nbytes}", gb, rs_rand)
        for op in ("AVG", "PRODUCT", "MAX", "MIN"):
            n = (64 << 10) // 4
            lo, hi = (0.9, 1.1) if op == "PRODUCT" else (-1.0, 1.0)

            def ar_op(op=op, n=n, lo=lo, hi=hi):
                xs = [_seeded((n,), f32, 99 + r, dev, lo, hi) for r in range(W)]
                t = xs[rank].clone()
                dist.all_reduce(t, op=getattr(dist.ReduceOp, op), group=g)
                return _close(t, xs, op, W, "float32")

            P.check(f"random/{eng}/all_reduce/float32/{op}/{n * 4}", gb, ar_op)

        # ---- async then sync on one tensor, and two same-member groups interleaved
        def async_then_sync():
            n = (1 << 20) // 4 if max_bytes >= (1 << 20) else 1024
            x = torch.full((n,), float(rank + 1), device=dev)
            w = dist.all_reduce(x, group=g, async_op=True)
            dist.all_reduce(x, group=g)
            w.wait()
            return bool(torch.all(x == W * (W + 1) / 2 * W).item())

        def shared_comm():
            n = 4096
            a = [torch.full((n,), float(rank + 1 + 10 * i), device=dev) for i in range(3)]
            b = [torch.full((n,), float(rank + 1 + 10 * i), device=dev) for i in range(3)]
            ws = []
            for i in range(3):
                ws.append(dist.all_reduce(a[i], group=g, async_op=True))
                dist.all_reduce(b[i], group=g2)
            for w in ws:
                w.wait()
            want = [W * (W + 1) / 2 + 10 * i * W for i in range(3)]
            return all(bool(torch.all(a[i] == want[i]).item()) and bool(torch.all(b[i] == want[i]).item())
                       for i in range(3))

        P.check(f"async_then_sync/{eng}", gb, async_then_sync)
        P.check(f"shared_comm/{eng}", gb2, shared_comm)

    # ---- protocol-specific paths of the peer-memory engine
    if on_gpu and world > 1 and ipc_ok:
        set_engine("ipc")
        if ll_ok:
            n = 1024  # 4 KiB of fp32
            root = W - 1

            def ll_all_reduce():
                xs = [_seeded((n,), f32, 500 + r, dev) for r in range(W)]
                t = xs[rank].clone()
                dist.all_reduce(t, group=g)
                return _close(t, xs, "SUM", W, "float32")

            def ll_reduce():
                xs = [_seeded((n,), f32, 600 + r, dev) for r in range(W)]
                t = xs[rank].clone()
                dist.reduce(t, dst=root, group=g)
                return _close(t, xs, "SUM", W, "float32") if rank == root else bool(torch.equal(t, xs[rank]))

            def ll_broadcast():
                src = _seeded((n,), f32, 700, dev)
                t = src.clone() if rank == root else torch.zeros(n, device=dev)
                dist.broadcast(t, src=root, group=g)
                return bool(torch.equal(t, src))

            def ll_all_gather():
                xs = [_seeded((n,), f32, 800 + r, dev) for r in range(W)]
                lst = [torch.empty(n, device=dev) for _ in range(W)]
                dist.all_gather(lst, xs[rank], group=g)
                return all(bool(torch.equal(lst[r], xs[r])) for r in range(W))

            def ll_gather():
                xs = [_seeded((n,), f32, 900 + r, dev) for r in range(W)]
                lst = [torch.empty(n, device=dev) for _ in range(W)] if rank == 0 else []
                dist.gather(xs[rank], gather_list=lst, dst=0, group=g)
                return rank != 0 or all(bool(torch.equal(lst[r], xs[r])) for r in range(W))

            def ll_scatter():
                xs = [_seeded((n,), f32, 1000 + r, dev) for r in range(W)]
                t = torch.empty(n, device=dev)
                dist.scatter(t, scatter_list=xs if rank == 0 else [], src=0, group=g)
                return bool(torch.equal(t, xs[rank]))

            def ll_reduce_scatter():
                xs = [[_seeded((n,), f32, 1100 + 10 * r + q, dev) for q in range(W)] for r in range(W)]
                out = torch.empty(n, device=dev)
                dist.reduce_scatter(out, [x.clone() for x in xs[rank]], group=g)
                return _close(out, [xs[r][rank] for r in range(W)], "SUM", W, "float32")

            def ll_all_to_all():
                xs = [[_seeded((n,), f32, 1200 + 10 * r + q, dev) for q in range(W)] for r in range(W)]
                outs = [torch.empty(n, device=dev) for _ in range(W)]
                dist.all_to_all(outs, xs[rank], group=g)
                return all(bool(torch.equal(outs[q], xs[q][rank])) for q in range(W))

            for name, fn in (("all_reduce", ll_all_reduce), ("reduce", ll_reduce), ("broadcast", ll_broadcast),
                             ("all_gather", ll_all_gather), ("gather", ll_gather), ("scatter", ll_scatter),
                             ("reduce_scatter", ll_reduce_scatter), ("all_to_all_list", ll_all_to_all)):
                P.check(f"ll/{name}", gb, fn, expect_engine="ipc_ll")
        if zc_ok and max_bytes >= (4 << 20):
            n = (4 << 20) // 4

            def zc_all_reduce():
                xs = [_seeded((n,), f32, 1300 + r, dev) for r in range(W)]
                t = xs[rank].clone()
                dist.all_reduce(t, group=g)
                return _close(t, xs, "SUM", W, "float32")

            # (per-rank payloads of 4 MiB at every W: the zero-copy threshold, PDCC_IPC_ZC_MIN = 1 MiB,
            # applies to one rank's input / output chunk -- 4 MiB / W would run staged from W = 5 on)
            def zc_all_gather():
                xs = [_seeded((n,), f32, 1400 + r, dev) for r in range(W)]
                out = torch.empty(n * W, device=dev)
                dist.all_gather_into_tensor(out, xs[rank], group=g)
                return bool(torch.equal(out, torch.cat(xs)))

            def zc_reduce_scatter():
                xs = [_seeded((n * W,), f32, 1500 + r, dev) for r in range(W)]
                out = torch.empty(n, device=dev)
                dist.reduce_scatter_tensor(out, xs[rank], group=g)
                return _close(out, [x[rank * n:(rank + 1) * n] for x in xs], "SUM", W, "float32")

            def zc_broadcast():
                src = _seeded((n,), f32, 1600, dev)
                t = src.clone() if rank == 0 else torch.zeros(n, device=dev)
                dist.broadcast(t, src=0, group=g)
                return bool(torch.equal(t, src))

            P.check("zc/all_reduce_pull", gb, zc_all_reduce, expect_engine="ipc_2shot_zc")
            P.check("zc/all_gather", gb, zc_all_gather, expect_engine="ipc_zc")
            P.check("zc/reduce_scatter", gb, zc_reduce_scatter, expect_engine="ipc_zc")
            P.check("zc/broadcast", gb, zc_broadcast, expect_engine="ipc_2shot_zc")
            set_engine("ipc_push")
            P.check("zc/all_reduce_push", gb, zc_all_reduce, expect_engine="ipc_push_zc")
            set_engine("ipc_dyn")
            P.check("zc/all_reduce_dyn", gb, zc_all_reduce, expect_engine="ipc_2shot_dyn_zc")
            # every other engine the autotuner can adopt for a key, forced (verdict r4 Next #1):
            # the dynamic all-gather / reduce-scatter, the staged (no zero copy) protocols, the
            # wide-grid pull all-reduce and -- where RCCL runs -- the wide RCCL communicator
            P.check("dyn/all_gather", gb, zc_all_gather, expect_engine="ipc_dyn_zc")
            P.check("dyn/reduce_scatter", gb, zc_reduce_scatter, expect_engine="ipc_dyn_zc")
            set_engine("ipc_staged")
            P.check("staged/all_reduce", gb, zc_all_reduce, expect_engine="ipc_2shot")
            P.check("staged/all_gather", gb, zc_all_gather, expect_engine="ipc")
            P.check("staged/reduce_scatter", gb, zc_reduce_scatter, expect_engine="ipc")
            P.check("staged/broadcast", gb, zc_broadcast, expect_engine="ipc_2shot")
            set_engine("ipc_wide")
            P.check("wide/all_reduce", gb, zc_all_reduce, expect_engine="ipc_2shot_wide*")
            _sdma_checks(P, g, gb, set_engine, rank, W, dev, n)
            if rccl_ok:
                set_engine("rccl_wide")
                P.check("rccl_wide/all_reduce", gb, zc_all_reduce, expect_engine="rccl_wide")
    if on_gpu and (world > 1 or rccl_ok):
        # verdict r5 Next #2: the custom ReduceOps at zero-copy / bulk sizes through every engine that
        # can serve them (BASELINE.json configs[4]), and RCCL's bulk reduce leaving non-roots untouched
        eng = [("rccl", "rccl*")] if rccl_ok else []
        if world > 1 and ipc_ok:
            eng += ([("ipc", "ipc_2shot_zc"), ("ipc_dyn", "ipc_2shot_dyn_zc"), ("ipc_push", "ipc_push_zc"),
                     ("ipc_staged", "ipc_2shot")] if zc_ok else [("ipc", "ipc_2shot")])
        sizes = [b for b in (4 << 20, 64 << 20) if b <= max_bytes]
        if not sizes:  # a small rehearsal (PDCC_BENCH_SMALL): RCCL's variants at the size it has
            eng, sizes = [e for e in eng if e[0] == "rccl"], [max_bytes]
        _op_checks(P, g, gb, set_engine, rank, W, dev, eng, sizes)
    if on_gpu and world > 1:
        _coalesced_checks(P, g, gb, set_engine, rank, W, dev, ("ipc",) * ipc_ok + ("rccl",) * rccl_ok)
        if ipc_ok:
            _async_capped_checks(P, rank, W, dev, to, zc_ok and max_bytes >= (4 << 20))
        if ipc_ok and max_bytes >= (16 << 20):
            set_engine("auto")
            _raced_key_checks(P, g, gb, rank, W, dev, rccl_ok, zc_ok)
    set_engine("auto")
    out = P.result()
    out["info"] = info
    for grp in (g2, g):
        try:
            dist.destroy_process_group(grp)
        except Exception:
            pass
    return out


def _sdma_checks(P, g, gb, set_engine, rank, W, dev, n):
    """The copy-engine engine (``ipc_sdma``: hipMemcpyAsync pulls between IPC-mapped user buffers), forced,
    for every copy collective at a zero-copy size (`n` fp32 per rank), bitwise against the inputs."""
    import torch
    import torch.distributed as dist

    f32 = torch.float32
    set_engine("ipc_sdma")

    def bcast():
        src = _seeded((n,), f32, 1700, dev)
        t = src.clone() if rank == 0 else torch.zeros(n, device=dev)
        dist.broadcast(t, src=0, group=g)
        return bool(torch.equal(t, src))

    def ag_flat():
        xs = [_seeded((n,), f32, 1710 + r, dev) for r in range(W)]
        out = torch.empty(n * W, device=dev)
        dist.all_gather_into_tensor(out, xs[rank], group=g)
        return bool(torch.equal(out, torch.cat(xs)))

    def ag_list():
        xs = [_seeded((n,), f32, 1720 + r, dev) for r in range(W)]
        outs = [torch.empty(n + 64, device=dev)[:n] for _ in range(W)]  # never adjacent
        dist.all_gather(outs, xs[rank], group=g)
        return all(bool(torch.equal(outs[r], xs[r])) for r in range(W))

    def gather():
        xs = [_seeded((n,), f32, 1730 + r, dev) for r in range(W)]
        outs = [torch.empty(n, device=dev) for _ in range(W)] if rank == W - 1 else None
        dist.gather(xs[rank], gather_list=outs, dst=W - 1, group=g)
        return rank != W - 1 or all(bool(torch.equal(outs[r], xs[r])) for r in range(W))

    def scatter():
        flat = _seeded((n * W,), f32, 1740, dev)
        out = torch.empty(n, device=dev)
        dist.scatter(out, scatter_list=list(flat.chunk(W)) if rank == 0 else None, src=0, group=g)
        return bool(torch.equal(out, flat[rank * n:(rank + 1) * n]))

    def a2a():
        xs = [_seeded((n * W,), f32, 1750 + r, dev) for r in range(W)]
        out = torch.empty(n * W, device=dev)
        dist.all_to_all_single(out, xs[rank], group=g)
        return bool(torch.equal(out, torch.cat([x[rank * n:(rank + 1) * n] for x in xs])))

    for name, fn in (("broadcast", bcast), ("all_gather", ag_flat), ("all_gather_list", ag_list),
                     ("gather", gather), ("scatter", scatter), ("all_to_all", a2a)):
        P.check(f"sdma/{name}", gb, fn, expect_engine="ipc_sdma_zc")
    set_engine("ipc")


def _op_checks(P, g, gb, set_engine, rank, W, dev, engines, sizes):
    """PRODUCT / MAX / MIN / AVG fp32 all_reduce of seeded data per (engine, size) against an fp64
    reduction of every rank's input (MAX / MIN bitwise), the engine required to be the one forced
    (zero-copy ones: no call of the check may have run staged); RCCL's bulk reduce: root within
    tolerance, every other rank's buffer bit-identical to its input."""
    import torch
    import torch.distributed as dist

    f32 = torch.float32
    for name, want in engines:
        set_engine(name)
        for nbytes in sizes:
            n = nbytes // 4
            for op in ("PRODUCT", "MAX", "MIN", "AVG"):
                lo, hi = (0.9, 1.1) if op == "PRODUCT" else (-1.0, 1.0)

                def ar_op(op=op, n=n, lo=lo, hi=hi, seed=3000 + nbytes % 997):
                    xs = [_seeded((n,), f32, seed + r, dev, lo, hi) for r in range(W)]
                    t = xs[rank].clone()
                    dist.all_reduce(t, op=getattr(dist.ReduceOp, op), group=g)
                    return _close(t, xs, op, W, "float32")

                P.check(f"ops/{name}/all_reduce/{op}/{nbytes >> 20}MiB", gb, ar_op, expect_engine=want)
        if name == "rccl" and sizes:
            n = sizes[-1] // 4

            def rd_bulk(n=n):
                xs = [_seeded((n,), f32, 4100 + r, dev) for r in range(W)]
                t = xs[rank].clone()
                dist.reduce(t, dst=0, group=g)
                return _close(t, xs, "SUM", W, "float32") if rank == 0 else bool(torch.equal(t, xs[rank]))

            P.check(f"ops/rccl/reduce/SUM/{sizes[-1] >> 20}MiB_nonroot_untouched", gb, rd_bulk, expect_engine="rccl*")
    set_engine("auto")


def _capped_count(gb) -> int:
    import re

    m = re.search(r"async_capped=(\d+)", gb.describe())
    return int(m.group(1)) if m else 0


def _coalesced_checks(P, g, gb, set_engine, rank, W, dev, engines):
    """The three coalesced collectives (DDP / ZeRO buckets: one collective per call,
    csrc/backend/coalesced.cpp) with 64 ragged fp32 members, per engine, against fp64."""
    import torch
    import torch.distributed as dist

    from .. import distributed as pdist

    f32 = torch.float32
    sizes = [4096 + 13 * i + (i % 3) for i in range(64)]  # ragged: not multiples of 16 B

    def member(i, r, salt=0):
        return _seeded((sizes[i],), f32, 20000 + 7919 * salt + 101 * i + r, dev)

    for eng in engines:
        set_engine(eng)
        want = eng + "*"

        def ar():
            ts = [member(i, rank).clone() for i in range(64)]
            dist.all_reduce_coalesced(ts, group=g)
            return all(_close(ts[i], [member(i, r) for r in range(W)], "SUM", W, "float32") for i in range(64))

        def ag():
            ins = [member(i, rank, 1) for i in range(64)]
            outs = [torch.empty(W * sizes[i], device=dev) for i in range(64)]
            pdist.all_gather_into_tensor_coalesced(outs, ins, group=g)
            return all(bool(torch.equal(outs[i], torch.cat([member(i, r, 1) for r in range(W)]))) for i in range(64))

        def rs():
            ins = [torch.cat([member(i, 100 * rank + q, 2) for q in range(W)]) for i in range(64)]
            outs = [torch.empty(sizes[i], device=dev) for i in range(64)]
            pdist.reduce_scatter_tensor_coalesced(outs, ins, group=g)
            return all(_close(outs[i], [member(i, 100 * r + rank, 2) for r in range(W)], "SUM", W, "float32")
                       for i in range(64))

        P.check(f"coalesced/{eng}/all_reduce_x64", gb, ar, expect_engine=want)
        P.check(f"coalesced/{eng}/all_gather_x64", gb, ag, expect_engine=want)
        P.check(f"coalesced/{eng}/reduce_scatter_x64", gb, rs, expect_engine=want)
    set_engine("auto")


def _async_capped_checks(P, rank, W, dev, to, zc):
    """async_op=True collectives on a group built with the (opt-in) async grid cap: the IPC
    launches run PDCC_IPC_ASYNC_GRID=64 workgroups (counted in describe(): async_capped);
    pull 2-shot and dynamic all-reduce, waited and checked against fp64."""
    import os

    import torch
    import torch.distributed as dist

    from ..parallel import backend as be

    saved = os.environ.get("PDCC_IPC_ASYNC_GRID")
    os.environ["PDCC_IPC_ASYNC_GRID"] = "64"  # read once, when the group's backend is built
    try:
        g3 = dist.new_group(list(range(W)), timeout=to)
    finally:
        if saved is None:
            os.environ.pop("PDCC_IPC_ASYNC_GRID", None)
        else:
            os.environ["PDCC_IPC_ASYNC_GRID"] = saved
    gb3 = be.native_backend(g3, dev.type)
    n = ((4 << 20) if zc else (256 << 10)) // 4 + 5  # + a ragged staged rest
    for eng, want in (("ipc", "ipc_*"), ("ipc_dyn", "ipc_2shot_dyn*" if zc else "ipc_*")):
        gb3.set_algo(eng)

        def fn(eng=eng):
            xs = [_seeded((n,), torch.float32, 30000 + 13 * len(eng) + r, dev) for r in range(W)]
            t = xs[rank].clone()
            c0 = _capped_count(gb3)
            dist.all_reduce(t, group=g3, async_op=True).wait()
            return _close(t, xs, "SUM", W, "float32") and _capped_count(gb3) > c0

        P.check(f"async_capped/{eng}/all_reduce", gb3, fn, expect_engine=want)
    try:
        dist.destroy_process_group(g3)
    except Exception:
        pass


def _raced_key_checks(P, g, gb, rank, W, dev, rccl_ok, zc_ok):
    """Autotuned bulk keys (the 1 GiB headline's race, at 24 MiB): the table row must list
    every candidate engine as raced (a time > 0) and valid (its sample matched the
    reference engine's on every rank), and the call's result must be right. Also an
    int32 BXOR key (no RCCL reduction exists: the static IPC engine is the reference,
    itself checked against the host transport on a prefix)."""
    import functools

    import torch
    import torch.distributed as dist

    def row_for(coll, dtype, op, nbytes):
        for e in gb.autotune_table():
            if e["coll"] == coll and e["dtype"] == dtype and e["op"] == op and e["lo"] <= nbytes < e["hi"]:
                return e
        return None

    n = (24 << 20) // 4

    def f32_sum():
        xs = [_seeded((n,), torch.float32, 40000 + r, dev) for r in range(W)]
        t = xs[rank].clone()
        dist.all_reduce(t, group=g)
        e = row_for("allreduce", "Float", "SUM", n * 4)
        if e is None or not e["ipc_valid"]:
            return False
        # (a wide RCCL child the runtime refused leaves the race on every rank: rccl_wide_ctas=0)
        wide = rccl_ok and "rccl_wide_ctas=0 " not in gb.describe()
        raced = ["ipc_us"] + (["wide_us"] if wide else []) + (["ipc_wide_us"] if rccl_ok else []) + \
                (["staged_us", "push_us", "dyn_us"] if zc_ok else [])
        if e["ref"] != ("rccl" if rccl_ok else "ipc") or any(e[k] <= 0 for k in raced + ["ref_us"]):
            return False
        return _close(t, xs, "SUM", W, "float32")

    def i32_bxor():
        def seeded_int(r):
            gen = torch.Generator(device=dev).manual_seed(50000 + r)
            return torch.randint(0, 1 << 30, (n,), generator=gen, device=dev, dtype=torch.int32)

        xs = [seeded_int(r) for r in range(W)]
        t = xs[rank].clone()
        dist.all_reduce(t, op=dist.ReduceOp.BXOR, group=g)
        e = row_for("allreduce", "Int", "BXOR", n * 4)
        if e is None or not e["ipc_valid"] or e["ref"] != "ipc" or e["ipc_us"] <= 0:
            return False
        if zc_ok and any(e[k] <= 0 for k in ("staged_us", "push_us", "dyn_us")):
            return False
        return bool(torch.equal(t, functools.reduce(torch.bitwise_xor, xs)))

    P.check("raced/all_reduce/float32/SUM/24MiB", gb, f32_sum, expect_engine="*")
    P.check("raced/all_reduce/int32/BXOR/24MiB", gb, i32_bxor, expect_engine="ipc*")
