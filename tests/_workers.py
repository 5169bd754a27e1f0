"""Per-rank worker functions for the multi-process tests (picklable by name).

Each returns plain Python data; the test process compares it with the golden
values of the reference (README.md:105-284 outputs).
"""
from __future__ import annotations

import os
import time


def _dev(device: str):
    import torch

    if device == "cpu":
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def golden(rank, size, device="cpu", subgroup=True):
    """The six primitives exactly as the reference calls them (main.py:9-83)."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    g = dist.new_group(list(range(size))) if subgroup else None
    out = {}
    t = torch.ones(1, device=d)
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM, group=g)
    out["reduce"] = t.cpu().tolist()
    t = torch.ones(1, device=d)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=g)
    out["all_reduce"] = t.cpu().tolist()
    t = torch.empty(1, device=d)
    if rank == 0:
        dist.scatter(t, scatter_list=[torch.tensor([i + 1.0], device=d) for i in range(size)], src=0, group=g)
    else:
        dist.scatter(t, scatter_list=[], src=0, group=g)
    out["scatter"] = t.cpu().tolist()
    t = torch.tensor([float(rank)], device=d)
    if rank == 0:
        lst = [torch.empty(1, device=d) for _ in range(size)]
        dist.gather(t, gather_list=lst, dst=0, group=g)
        out["gather"] = [x.item() for x in lst]
    else:
        dist.gather(t, gather_list=[], dst=0, group=g)
    lst = [torch.empty(1, device=d) for _ in range(size)]
    dist.all_gather(lst, torch.tensor([float(rank)], device=d), group=g)
    out["all_gather"] = [x.item() for x in lst]
    t = torch.tensor([0.0], device=d) if rank == 0 else torch.empty(1, device=d)
    dist.broadcast(t, src=0, group=g)
    out["broadcast"] = t.cpu().tolist()
    return out


def expected_golden(rank, size):
    e = {
        "all_reduce": [float(size)],
        "scatter": [rank + 1.0],
        "all_gather": [float(r) for r in range(size)],
        "broadcast": [0.0],
    }
    if rank == 0:
        e["reduce"] = [float(size)]
        e["gather"] = [float(r) for r in range(size)]
    else:
        # non-root reduce buffers are left untouched (Gloo's 3,2,1 leftovers in
        # README.md:106-109 are an implementation artifact, not a contract)
        e["reduce"] = [1.0]
    return e


def op_matrix(rank, size, device="cpu", dtypes=("float32", "float64", "int32", "int64", "bfloat16", "float16")):
    """all_reduce and reduce for every ReduceOp x dtype with t=[r+2, 10-r, r]
    (the survey's probe)."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    res = {}
    for dt in dtypes:
        tdt = getattr(torch, dt)
        for op in ("SUM", "PRODUCT", "MAX", "MIN", "AVG"):
            if op == "AVG" and not tdt.is_floating_point:
                continue
            t = torch.tensor([rank + 2, 10 - rank, rank], dtype=tdt, device=d)
            dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
            res[f"all_reduce/{dt}/{op}"] = t.float().cpu().tolist()
            t = torch.tensor([rank + 2, 10 - rank, rank], dtype=tdt, device=d)
            dist.reduce(t, dst=size - 1, op=getattr(dist.ReduceOp, op))
            if rank == size - 1:
                res[f"reduce/{dt}/{op}"] = t.float().cpu().tolist()
        if not tdt.is_floating_point:
            for op in ("BAND", "BOR", "BXOR"):
                t = torch.tensor([rank + 2, 10 - rank, rank], dtype=tdt, device=d)
                dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
                res[f"all_reduce/{dt}/{op}"] = t.float().cpu().tolist()
    return res


def expected_op(size, op):
    import functools

    vals = [[r + 2, 10 - r, r] for r in range(size)]
    cols = list(zip(*vals))
    f = {
        "SUM": sum,
        "PRODUCT": lambda c: functools.reduce(lambda a, b: a * b, c),
        "MAX": max,
        "MIN": min,
        "AVG": lambda c: sum(c) / len(c),
        "BAND": lambda c: functools.reduce(lambda a, b: a & b, c),
        "BOR": lambda c: functools.reduce(lambda a, b: a | b, c),
        "BXOR": lambda c: functools.reduce(lambda a, b: a ^ b, c),
    }[op]
    return [float(f(c)) for c in cols]


def large(rank, size, device="cpu", n=3_000_017):
    """Bulk paths (chunking across shm slots / IPC staging, tails not multiple of 16 B)."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    ok = {}
    base = torch.arange(n, dtype=torch.float32, device=d) % 1000
    t = base * (rank + 1)
    dist.all_reduce(t)
    ok["all_reduce"] = bool(torch.equal(t, base * (size * (size + 1) // 2)))
    t = base * (rank + 1)
    dist.reduce(t, dst=0)
    ok["reduce"] = bool(torch.equal(t, base * (size * (size + 1) // 2))) if rank == 0 else bool(torch.equal(t, base * (rank + 1)))
    t = base.clone() if rank == 0 else torch.zeros_like(base)
    dist.broadcast(t, src=0)
    ok["broadcast"] = bool(torch.equal(t, base))
    m = n // 7 + 3
    lst = [torch.empty(m, dtype=torch.float32, device=d) for _ in range(size)]
    dist.all_gather(lst, torch.full((m,), float(rank), device=d))
    ok["all_gather"] = all(bool(torch.all(x == r)) for r, x in enumerate(lst))
    o = torch.empty(size * m, device=d)
    dist.all_gather_into_tensor(o, torch.full((m,), float(rank), device=d))
    ok["all_gather_into_tensor"] = bool(torch.equal(o, torch.arange(size, device=d).float().repeat_interleave(m)))
    inp = torch.arange(size * m, dtype=torch.float32, device=d) % 97
    o = torch.empty(m, device=d)
    dist.reduce_scatter_tensor(o, inp)
    ok["reduce_scatter_tensor"] = bool(torch.equal(o, (inp * size)[rank * m:(rank + 1) * m]))
    ins = [torch.full((m,), float(rank * 100 + q), device=d) for q in range(size)]
    outs = [torch.empty(m, device=d) for _ in range(size)]
    dist.all_to_all(outs, ins)
    ok["all_to_all"] = all(bool(torch.all(outs[q] == q * 100 + rank)) for q in range(size))
    x = torch.arange(size * 5, dtype=torch.float32, device=d) + 1000 * rank
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    exp = torch.cat([torch.arange(rank * 5, rank * 5 + 5, dtype=torch.float32) + 1000 * q for q in range(size)])
    ok["all_to_all_single"] = bool(torch.equal(y.cpu(), exp))
    # uneven splits: rank r sends (q+1) rows to q
    in_splits = [q + 1 for q in range(size)]
    out_splits = [rank + 1] * size
    x = torch.cat([torch.full((q + 1, 3), float(rank * 10 + q)) for q in range(size)]).to(d)
    y = torch.empty(sum(out_splits), 3, device=d)
    dist.all_to_all_single(y, x, out_splits, in_splits)
    exp = torch.cat([torch.full((rank + 1, 3), float(q * 10 + rank)) for q in range(size)])
    ok["all_to_all_single_uneven"] = bool(torch.equal(y.cpu(), exp))
    dist.barrier()
    return ok


def noncontig(rank, size, device="cpu"):
    import torch
    import torch.distributed as dist

    d = _dev(device)
    a = torch.arange(64, dtype=torch.float32, device=d).reshape(8, 8) * (rank + 1)
    v = a.t()  # non-contiguous view
    dist.all_reduce(v)
    s = size * (size + 1) // 2
    ok1 = bool(torch.equal(a, torch.arange(64, dtype=torch.float32, device=d).reshape(8, 8) * s))
    b = (torch.arange(20, dtype=torch.float32, device=d) + rank)[1:]  # misaligned view (offset 4 B)
    dist.all_reduce(b)
    ok2 = bool(torch.equal(b, (torch.arange(20, dtype=torch.float32, device=d) * size + s - size)[1:]))
    return {"transposed": ok1, "offset": ok2}


def subgroup_evens(rank, size, device="cpu"):
    import torch
    import torch.distributed as dist

    evens = list(range(0, size, 2))
    g = dist.new_group(evens)
    t = torch.tensor([float(rank)], device=_dev(device))
    if rank in evens:
        dist.all_reduce(t, group=g)
    return t.item()


def p2p(rank, size, device="cpu", n=600_000):
    """Ring exchange with isend/irecv larger than the p2p channel, then a batch."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    nxt, prv = (rank + 1) % size, (rank - 1) % size
    x = torch.full((n,), float(rank), device=d)
    y = torch.empty(n, device=d)
    s = dist.isend(x, nxt)
    r = dist.irecv(y, prv)
    s.wait()
    r.wait()
    ok1 = bool(torch.all(y == prv))
    y2 = torch.empty(n, device=d)
    ops = [dist.P2POp(dist.isend, x * 2, nxt), dist.P2POp(dist.irecv, y2, prv)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    ok2 = bool(torch.all(y2 == 2 * prv))
    return {"ring": ok1, "batch": ok2}


def errors(rank, size):
    """Argument errors must raise on every rank (SURVEY.md §4.2 error contracts)."""
    import torch
    import torch.distributed as dist

    msgs = {}
    try:
        dist.broadcast(torch.ones(1), src=size)
    except (RuntimeError, ValueError) as e:
        msgs["bad_root"] = str(e)
    try:
        dist.all_gather([torch.empty(1) for _ in range(size + 1)], torch.ones(1))
    except (RuntimeError, ValueError) as e:
        msgs["bad_list"] = str(e)
    # the group is still usable afterwards
    t = torch.ones(1)
    dist.all_reduce(t)
    msgs["after"] = t.item()
    return msgs


def debug_mismatch(rank, size):
    import torch
    import torch.distributed as dist

    t = torch.ones(4 + rank)  # per-rank shape mismatch: silent with Gloo on rank 0
    try:
        dist.all_reduce(t)
        return "no error"
    except RuntimeError as e:
        return str(e)


def stats_probe(rank, size):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend

    t = torch.ones(16)
    dist.all_reduce(t)
    st = backend.stats()
    zc = dict(backend.native_backend(None, "cpu").zc_counters())  # (no GPU op: every counter 0)
    return {k: list(v) for k, v in st.items()}, backend.describe(), zc, backend.last_algo()


def timing_allreduce(rank, size, n=1 << 20, iters=20):
    import torch
    import torch.distributed as dist

    t = torch.ones(n)
    dist.all_reduce(t)
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(t)
    return (time.perf_counter() - t0) / iters


def fault_victim(rank, size, q):
    """rank 1 dies (PDCC_FAULT=1:3:exit); rank 0 must get an error, fast."""
    import datetime

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel.spawn import init_process

    def body(r, s):
        t0 = time.time()
        try:
            for _ in range(50):
                x = torch.ones(8)
                dist.all_reduce(x)
            return ("no error", time.time() - t0)
        except RuntimeError as e:
            return (str(e), time.time() - t0)

    res = init_process(rank, size, body, timeout_s=60)
    q.put((rank, res))


def demo(rank, size, name, device="cpu"):
    from pytorch_distributed_collective_communication_amd.models.demos import DEMOS

    return DEMOS[name](rank, size, device)


def dp_train(rank, size, mode="bucketer", steps=5, device="cpu", bucket_bytes=2048):
    """Data-parallel SGD on the MLP; returns the flattened final parameters."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.models import MLP, synthetic_batch
    from pytorch_distributed_collective_communication_amd.parallel import ddp

    d = _dev(device)
    torch.manual_seed(100 + rank)  # deliberately different init: broadcast must fix it
    model = MLP().to(d)
    ddp.broadcast_parameters(model, src=0)
    x, y = synthetic_batch(64, device=d)
    shard = 64 // size
    xs, ys = x[rank * shard:(rank + 1) * shard], y[rank * shard:(rank + 1) * shard]
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    if mode == "torch_ddp":
        net = torch.nn.parallel.DistributedDataParallel(model)
    else:
        net = model
        buck = ddp.GradBucketer(model, bucket_bytes=bucket_bytes)
    for _ in range(steps):
        opt.zero_grad(set_to_none=False)
        loss = torch.nn.functional.mse_loss(net(xs), ys)
        loss.backward()
        if mode != "torch_ddp":
            buck.finish()
        opt.step()
    # plain floats: a torch tensor sent through an mp.Queue is shared by fd passing,
    # which races with this process exiting
    return torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]).tolist()


def dp_reference(steps=5):
    import torch

    from pytorch_distributed_collective_communication_amd.models import MLP, synthetic_batch

    torch.manual_seed(100)
    model = MLP()
    x, y = synthetic_batch(64)
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    for _ in range(steps):
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


def flight_probe(rank, size):
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend

    for n in (1, 10, 100):
        dist.all_reduce(torch.ones(n))
    dist.broadcast(torch.ones(3), 0)
    b = backend.native_backend()
    return b.flight_recorder(), b.flight_recorder_dump(3)


def two_groups(rank, size, device="cuda"):
    """Two process groups in one process, both on the IPC path, interleaved
    (regression: the second group's hipIpc mappings must not alias the first's)."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    g = dist.new_group(list(range(size)))
    ok = []
    for n in (1, 1000, 300_000):
        a = torch.full((n,), float(rank + 1), device=d)
        b = torch.full((n,), float(10 * (rank + 1)), device=d)
        for _ in range(3):
            dist.all_reduce(a)
            dist.all_reduce(b, group=g)
        s = size * (size + 1) / 2
        ok.append(bool(torch.all(a == s * size ** 2).item()) and bool(torch.all(b == 10 * s * size ** 2).item()))
    return ok


def staging_growth(rank, size, device="cuda", max_bytes=64 << 20):
    """all_reduce with sizes doubling from 4 KiB to `max_bytes` on the world
    group, then on a second group: every doubling regrows the IPC staging
    (regression: with ranks sharing a device, a fresh allocation could land on a
    just-closed peer import and hipIpcGetMemHandle refused to export it)."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    g = dist.new_group(list(range(size)))
    ok = []
    for grp in (None, g):
        n = 1024
        while n * 4 <= max_bytes:
            x = torch.full((n,), float(rank + 1), device=d)
            dist.all_reduce(x, group=grp)
            ok.append(bool(torch.all(x == size * (size + 1) / 2).item()))
            n *= 2
    return ok


def async_ordering(rank, size, device="cuda", rounds=20):
    """async_op=True collectives run on the backend's comm stream: the hand-off
    from the caller's stream (producer kernels still running) and back (Work.wait
    / is_completed polling / futures) must order correctly."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    ok = []
    m = torch.randn(1024, 1024, device=d)
    for i in range(rounds):
        x = torch.zeros(1 << 18, device=d)
        for _ in range(4):  # keep the caller's stream busy before the producer write lands
            m = torch.tanh(m @ m)
        x.add_(float(rank + 1 + i) + 0 * m[0, 0])
        w = dist.all_reduce(x, async_op=True)
        if i % 3 == 0:
            w.wait()
        elif i % 3 == 1:
            while not w.is_completed():
                pass
            w.wait()
        else:
            w.get_future().wait()
        exp = sum(r + 1 + i for r in range(size))
        ok.append(bool(torch.all(x == exp).item()))
    # several in flight at once, then wait them in reverse
    xs = [torch.full((1000 * (k + 1),), float(k + rank), device=d) for k in range(6)]
    ws = [dist.all_reduce(t, async_op=True) for t in xs]
    for w in reversed(ws):
        w.wait()
    for k, t in enumerate(xs):
        ok.append(bool(torch.all(t == sum(k + r for r in range(size))).item()))
    return ok


def autotune_probe(rank, size, device="cuda"):
    """all_reduce across the autotuner's size buckets: the first call of each
    bucket times both engines on scratch copies; every call must still return
    the right sum, and the decision table must be identical on all ranks."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    ok = []
    for dt in (torch.float32, torch.bfloat16):
        # (16 K + 64) fp32 elements: just above the LL range, the smallest tuned bucket
        for n in ((16 << 10) + 64, 1 << 18, 1 << 20, 4 << 20):
            x = (torch.arange(n, device=d) % 13).to(dt) + rank
            exp = ((torch.arange(n, device=d) % 13).float() * size + size * (size - 1) / 2)
            for _ in range(3):
                y = x.clone()
                dist.all_reduce(y)
                ok.append(bool(torch.allclose(y.float(), exp, rtol=1e-2 if dt == torch.bfloat16 else 0)))
    return {"ok": ok, "table": be.autotune_table()}


def autotune_all_colls(rank, size, device="cuda", n=1 << 16):
    """Every tunable collective once at a tunable size (256 KiB of fp32): each call
    must be right, and the table must get one row per (collective, dtype, op,
    layout) -- identical on every rank. Then the ADVICE r1 case: a float SUM
    bucket decided first, an int32 BAND of the same size afterwards (no RCCL op
    exists for BAND: the key must not inherit the float decision)."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    ok = {}
    base = torch.arange(n, device=d, dtype=torch.float32) % 97
    t = base + rank
    dist.all_reduce(t)
    ok["all_reduce"] = bool(torch.equal(t, base * size + size * (size - 1) / 2))
    t = base + rank
    dist.reduce(t, dst=size - 1)
    ok["reduce"] = rank != size - 1 or bool(torch.equal(t, base * size + size * (size - 1) / 2))
    t = base.clone() if rank == 0 else torch.zeros_like(base)
    dist.broadcast(t, src=0)
    ok["broadcast"] = bool(torch.equal(t, base))
    out = torch.empty(n * size, device=d)
    dist.all_gather_into_tensor(out, base + rank)
    ok["all_gather_flat"] = all(bool(torch.equal(out[r * n:(r + 1) * n], base + r)) for r in range(size))
    lst = [torch.empty(n + 64, device=d)[:n] for _ in range(size)]  # gaps: never adjacent views
    dist.all_gather(lst, base + rank)
    ok["all_gather_list"] = all(bool(torch.equal(lst[r], base + r)) for r in range(size))
    glist = [torch.empty(n, device=d) for _ in range(size)] if rank == 0 else None
    dist.gather(base + rank, gather_list=glist, dst=0)
    ok["gather"] = rank != 0 or all(bool(torch.equal(glist[r], base + r)) for r in range(size))
    slist = [base + 1000 * r for r in range(size)] if rank == 0 else None
    so = torch.empty(n, device=d)
    dist.scatter(so, scatter_list=slist, src=0)
    ok["scatter"] = bool(torch.equal(so, base + 1000 * rank))
    inp = torch.cat([base + r for r in range(size)]) * (rank + 1)
    rs = torch.empty(n, device=d)
    dist.reduce_scatter_tensor(rs, inp)
    ok["reduce_scatter"] = bool(torch.equal(rs, (base + rank) * (size * (size + 1) / 2)))
    a2a_in = torch.cat([base + 100 * rank + q for q in range(size)])
    a2a_out = torch.empty_like(a2a_in)
    dist.all_to_all_single(a2a_out, a2a_in)
    ok["all_to_all"] = all(bool(torch.equal(a2a_out[q * n:(q + 1) * n], base + 100 * q + rank)) for q in range(size))
    # same size bucket, different dtype/op
    m = 25_600  # 100 KiB of fp32 / int32
    f = torch.full((m,), float(rank + 1), device=d)
    dist.all_reduce(f)
    ok["float_sum_100k"] = bool(torch.all(f == size * (size + 1) / 2))
    bits = torch.full((m,), (1 << rank) | 0x100, device=d, dtype=torch.int32)
    dist.all_reduce(bits, op=dist.ReduceOp.BAND)
    ok["int_band_100k"] = bool(torch.all(bits == 0x100))
    bits = torch.full((m,), 1 << rank, device=d, dtype=torch.int32)
    dist.all_reduce(bits, op=dist.ReduceOp.BOR)
    ok["int_bor_100k"] = bool(torch.all(bits == (1 << size) - 1))
    return {"ok": ok, "table": be.autotune_table()}


def group_churn(rank, size, device="cuda", groups=6):
    """The reference's pattern: a fresh new_group(range(size)) per demo
    (main.py:11,21,31,46,63,75), one collective in each. Returns per-group wall
    time of (new_group + first all_reduce) and how each group got its RCCL
    communicator (stats rows rccl_comm/<init|split|share>)."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    x = torch.ones(1024, device=d)
    t0 = time.perf_counter()
    dist.all_reduce(x)
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    ok = [bool(torch.all(x == size))]
    out = []
    for _ in range(groups):
        t0 = time.perf_counter()
        g = dist.new_group(list(range(size)))
        y = torch.ones(1024, device=d)
        dist.all_reduce(y, group=g)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok.append(bool(torch.all(y == size)))
        st = be.native_backend(g, "cuda").stats()
        how = sorted(k.split("/", 1)[1] for k in st if k.startswith("rccl_comm/"))
        setup_ms = sum(v[2] for k, v in st.items() if k.startswith("rccl_comm/"))
        out.append({"wall_ms": dt * 1e3, "how": how, "comm_ms": setup_ms})
    return {"ok": ok, "first_ms": first * 1e3, "groups": out}


def graph_capture(rank, size, device="cuda", replays=5):
    """Collectives captured into a hipGraph (parallel.graphs.capture) and replayed
    with new inputs each time, with an eager collective between two replays: the
    IPC kernels' device-side sequence numbers must keep every rank's flag epochs
    and staging parities in step across replays and eager calls."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel.graphs import capture

    d = _dev(device)
    small = torch.zeros(1000, device=d)      # IPC 1-shot
    mid = torch.zeros(300_000, device=d)     # 1.2 MB: IPC 2-shot (RCCL at world 1)
    bc = torch.zeros(5000, device=d)
    ag_in = torch.zeros(780, device=d)
    ag_out = torch.zeros(780 * size, device=d)

    def fill(i):
        small.fill_(float(rank + i))
        mid.fill_(float(2 * rank + i))
        bc.fill_(float(100 + i) if rank == 0 else -1.0)
        ag_in.fill_(float(10 * rank + i))

    def step():
        dist.all_reduce(small)
        dist.all_reduce(mid)
        dist.broadcast(bc, src=0)
        dist.all_gather_into_tensor(ag_out, ag_in)

    fill(0)
    g = capture(step, warmup=2)
    ok = []
    tri = size * (size - 1) / 2
    for i in range(1, replays + 1):
        fill(i)
        g.replay()
        if i == 3:  # an eager collective between two replays
            e = torch.full((4096,), float(rank), device=d)
            dist.all_reduce(e)
            ok.append(bool(torch.all(e == tri).item()))
        torch.cuda.synchronize()
        ok.append(bool(torch.all(small == tri + size * i).item()))
        ok.append(bool(torch.all(mid == 2 * tri + size * i).item()))
        ok.append(bool(torch.all(bc == 100 + i).item()))
        exp = torch.arange(size, device=d, dtype=torch.float32).repeat_interleave(780) * 10 + i
        ok.append(bool(torch.equal(ag_out, exp)))
    return ok


def ipc_selftest_probe(rank, size, device="cuda"):
    """One GPU all_reduce; returns (correct, whether the group kept the IPC path)."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    x = torch.full((1000,), float(rank + 1), device=_dev(device))
    dist.all_reduce(x)
    ok = bool(torch.all(x == size * (size + 1) / 2).item())
    return ok, "ipc_ok=1" in be.describe()


def gpu_fault_victim(rank, size, q, group_timeout_s=4):
    """Two ranks on the IPC path; rank 1 dies after setup. Rank 0's next GPU
    all_reduce spins in the cross-GPU barrier until the group timeout (bounded
    spin, error word), the watchdog poisons the group, and rank 0 gets a
    RuntimeError instead of a hang."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel.spawn import init_process

    def body(r, s):
        x = torch.ones(1 << 16, device="cuda")
        dist.all_reduce(x)  # IPC staging + peer mappings set up on both ranks
        torch.cuda.synchronize()
        dist.barrier()
        if r == 1:
            os._exit(13)
        time.sleep(0.5)
        t0 = time.time()
        try:
            for _ in range(3):
                dist.all_reduce(x)
                torch.cuda.synchronize()
                time.sleep(0.3)
            return ("no error", time.time() - t0)
        except RuntimeError as e:
            return (str(e), time.time() - t0)

    res = init_process(rank, size, body, bind_device=True, timeout_s=group_timeout_s)
    q.put((rank, res))


def p2p_subset(rank, size, device="cpu", n=300_000):
    """Point-to-point between two ranks of a larger group, issued before any
    collective: ranks 0 and 1 exchange (both directions, larger than a channel),
    the others do nothing until a later barrier. Then a ring of FIRST isends on
    a fresh group (each pair channel is built by the two ranks alone)."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    ok = {}
    if rank in (0, 1):
        peer = 1 - rank
        x = torch.full((n,), float(rank + 1), device=d)
        y = torch.empty(n, device=d)
        if rank == 0:
            dist.send(x, peer)
            dist.recv(y, peer)
        else:
            dist.recv(y, peer)
            dist.send(x, peer)
        ok["pair"] = bool(torch.all(y == peer + 1))
    dist.barrier()
    g = dist.new_group(list(range(size)))
    nxt, prv = (rank + 1) % size, (rank - 1) % size
    x = torch.full((n,), float(10 + rank), device=d)
    y = torch.empty(n, device=d)
    s = dist.isend(x, nxt, group=g)
    r = dist.irecv(y, prv, group=g)
    s.wait()
    r.wait()
    ok["ring_first_isend"] = bool(torch.all(y == 10 + prv))
    return ok


def dp_accum(rank, size, device="cpu", micro=2):
    """Gradient accumulation with GradBucketer.no_sync(): `micro` micro-batches per
    rank, one reduction per step; returns (params after one SGD step, whether a
    second backward without no_sync() raised)."""
    import torch

    from pytorch_distributed_collective_communication_amd.models import MLP, synthetic_batch
    from pytorch_distributed_collective_communication_amd.parallel import ddp

    d = _dev(device)
    torch.manual_seed(100 + rank)
    model = MLP().to(d)
    ddp.broadcast_parameters(model, src=0)
    x, y = synthetic_batch(64, device=d)
    shard = 64 // size
    xs, ys = x[rank * shard:(rank + 1) * shard], y[rank * shard:(rank + 1) * shard]
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    buck = ddp.GradBucketer(model, bucket_bytes=2048)
    opt.zero_grad(set_to_none=False)
    mb = shard // micro
    for k in range(micro):
        loss = torch.nn.functional.mse_loss(model(xs[k * mb:(k + 1) * mb]), ys[k * mb:(k + 1) * mb]) / micro
        if k < micro - 1:
            with buck.no_sync():
                loss.backward()
        else:
            loss.backward()
    buck.finish()
    opt.step()
    params = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]).tolist()
    raised = False
    try:
        for _ in range(2):
            torch.nn.functional.mse_loss(model(xs), ys).backward()
    except RuntimeError as e:
        raised = "no_sync" in str(e)
    return params, raised


def engine_crosscheck(rank, size, device="cuda"):
    """The same random inputs through RCCL and through the IPC kernels (forced per
    call with set_algo, identically on every rank): results must agree (SUM
    within summation-order rounding, MAX and the copy collectives exactly)."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    gen = torch.Generator(device=d).manual_seed(1000 + rank)
    ok = {}
    for n in (1000, 1 << 20, 3_000_017):
        x = torch.randn(n, generator=gen, device=d)
        res = {}
        for algo in ("rccl", "ipc"):
            b.set_algo(algo)
            y = x.clone()
            dist.all_reduce(y)
            m = x.clone()
            dist.all_reduce(m, op=dist.ReduceOp.MAX)
            lst = [torch.empty(n, device=d) for _ in range(size)]
            dist.all_gather(lst, x)
            res[algo] = (y, m, torch.cat(lst))
        b.set_algo("auto")
        ok[f"sum_{n}"] = bool(torch.allclose(res["rccl"][0], res["ipc"][0], rtol=1e-5, atol=1e-5 * size))
        ok[f"max_{n}"] = bool(torch.equal(res["rccl"][1], res["ipc"][1]))
        ok[f"all_gather_{n}"] = bool(torch.equal(res["rccl"][2], res["ipc"][2]))
    return ok


def eager_probe(rank, size, device="cuda"):
    """PDCC_EAGER_INIT=1: the RCCL communicator exists right after
    init_process_group (before the first collective), and collectives work."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    before = sorted(k for k in be.native_backend(None, "cuda").stats() if k.startswith("rccl_comm/"))
    x = torch.full((4096,), float(rank + 1), device=_dev(device))
    dist.all_reduce(x)
    return {"before": before, "ok": bool(torch.all(x == size * (size + 1) / 2))}


def autotune_fault_probe(rank, size, device="cuda"):
    """An IPC run of the autotune race that times out on one rank (rank 1 arrives
    late, PDCC_TEST_AUTOTUNE_DELAY) must disqualify IPC for that key only: the
    call still returns the right sum, the group stays healthy, and later calls
    (IPC included) work."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    x = torch.full((1 << 18,), float(rank + 1), device=d)  # 1 MiB: tuned bucket
    dist.all_reduce(x)
    ok = [bool(torch.all(x == size * (size + 1) / 2))]
    b = be.native_backend(None, "cuda")
    ok.append(b.healthy())
    y = torch.full((1000,), float(rank), device=d)  # small: IPC 1-shot by the static threshold
    dist.all_reduce(y)
    ok.append(bool(torch.all(y == size * (size - 1) / 2)))
    x.fill_(1.0)
    dist.all_reduce(x)
    ok.append(bool(torch.all(x == size)))
    return {"ok": ok, "table": be.autotune_table()}


def lifecycle_probe(rank, size, device="cpu"):
    """c10d lifecycle hooks: aborting a sub-group (ProcessGroup.abort ->
    Backend::abort) poisons it -- later calls fail fast with a clear error, getError
    reports it -- while the default group keeps working; destroy_process_group on a
    healthy group drains and shuts down cleanly."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    g = dist.new_group(list(range(size)))
    t = torch.ones(4, device=d)
    dist.all_reduce(t, group=g)
    ok = {"before": bool(torch.all(t == size))}
    g.abort()  # ProcessGroup.abort -> Backend::abort on every backend of the group
    try:
        dist.all_reduce(torch.ones(4, device=d), group=g)
        ok["after_abort_raises"] = False
    except RuntimeError as e:
        ok["after_abort_raises"] = "error state" in str(e) or "aborted" in str(e)
    t = torch.ones(4, device=d)
    dist.all_reduce(t)
    ok["default_group_alive"] = bool(torch.all(t == size))
    h = dist.new_group(list(range(size)))
    dist.all_reduce(t, group=h)
    dist.destroy_process_group(h)
    ok["healthy_flag"] = be.native_backend().healthy()
    return ok


def zero_copy(rank, size, device="cuda"):
    """Zero-copy IPC (PDCC_ALGO=ipc, PDCC_IPC_ZC on): the peers read each rank's own
    tensor in place. Sizes with and without a staged rest, one buffer reused (cached
    mappings), fresh allocations past the export cache with empty_cache() in between
    (eviction, allocations re-made at the same address), every zero-copy collective,
    and a rank-asymmetric layout (one rank's reduce_scatter input not flat: the group
    agrees to stage). Returns {check: bool}."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    ok = {}
    tile = 1024  # fp32 elements per 4 KiB tile
    tri = size * (size + 1) // 2
    for n in (size * tile * 300, size * tile * 300 + 77, (1 << 20) // 4 + 3, 3 * size * tile * 256 + 1):
        base = torch.arange(n, device=d, dtype=torch.float32) % 1000
        t = base * (rank + 1)
        dist.all_reduce(t)
        ok[f"all_reduce_{n}"] = bool(torch.equal(t, base * tri))
    x = torch.empty(size * tile * 256, device=d)
    for _ in range(10):
        x.fill_(rank + 1.0)
        dist.all_reduce(x)
    ok["reuse"] = bool(torch.all(x == tri))
    good = True
    for i in range(40):  # > PDCC_IPC_ZC_CACHE distinct allocations
        y = torch.full((tile * 512 + i * size * tile,), float(rank + i), device=d)
        dist.all_reduce(y)
        good = good and bool(torch.all(y == sum(r + i for r in range(size))))
        del y
        if i % 8 == 7:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    ok["churn"] = good
    m = tile * 300 + 5
    src = torch.full((m,), float(rank), device=d)
    out = torch.empty(size * m, device=d)
    dist.all_gather_into_tensor(out, src)
    ok["all_gather_into_tensor"] = bool(torch.equal(out, torch.arange(size, device=d).float().repeat_interleave(m)))
    lst = [torch.empty(m + 64, device=d)[:m] for _ in range(size)]
    dist.all_gather(lst, src)
    ok["all_gather_list"] = all(bool(torch.all(v == q)) for q, v in enumerate(lst))
    inp = torch.arange(size * m, dtype=torch.float32, device=d) % 97 + rank
    o = torch.empty(m, device=d)
    dist.reduce_scatter_tensor(o, inp)
    exp = ((torch.arange(size * m, dtype=torch.float32, device=d) % 97) * size + size * (size - 1) / 2)
    ok["reduce_scatter_tensor"] = bool(torch.equal(o, exp[rank * m:(rank + 1) * m]))
    a2a_in = torch.arange(size * m, dtype=torch.float32, device=d) + 10000 * rank
    a2a_out = torch.empty_like(a2a_in)
    dist.all_to_all_single(a2a_out, a2a_in)
    exp = torch.cat([torch.arange(rank * m, (rank + 1) * m, dtype=torch.float32, device=d) + 10000 * q
                     for q in range(size)])
    ok["all_to_all_single"] = bool(torch.equal(a2a_out, exp))
    b = torch.arange(size * tile * 200 + 9, dtype=torch.float32, device=d) if rank == 1 else \
        torch.zeros(size * tile * 200 + 9, device=d)
    dist.broadcast(b, src=1)
    ok["broadcast"] = bool(torch.equal(b, torch.arange(b.numel(), dtype=torch.float32, device=d)))
    for n in (size * tile * 300, size * tile * 300 + 77):  # rooted reduce: non-roots keep their input
        base = torch.arange(n, device=d, dtype=torch.float32) % 1000
        t = base * (rank + 1)
        dist.reduce(t, dst=size - 1)
        want = base * tri if rank == size - 1 else base * (rank + 1)
        ok[f"reduce_{n}"] = bool(torch.equal(t, want))
    sc_n = tile * 280 + 3
    for flat in (True, False):  # scatter from the root's list: flat views are read in place
        pool = torch.arange(size * sc_n, dtype=torch.float32, device=d)
        lst = list(pool.chunk(size)) if flat else [pool[q * sc_n:(q + 1) * sc_n].clone() for q in range(size)]
        o = torch.empty(sc_n, device=d)
        dist.scatter(o, scatter_list=lst if rank == 0 else None, src=0)
        ok[f"scatter_flat{int(flat)}"] = bool(torch.equal(o, pool[rank * sc_n:(rank + 1) * sc_n]))
    m2 = tile * 260
    full = torch.arange(size * m2, dtype=torch.float32, device=d)
    ins = list(full.chunk(size)) if rank == 0 else [full[q * m2:(q + 1) * m2].clone() for q in range(size)]
    o2 = torch.empty(m2, device=d)
    dist.reduce_scatter(o2, ins)
    ok["asymmetric_layout"] = bool(torch.equal(o2, full[rank * m2:(rank + 1) * m2] * size))
    st = be.stats()
    ok["zc_rows"] = any(k.endswith("_zc") for k in st)
    ok["zc_ok"] = "zc_ok=1" in be.describe()
    dist.barrier()
    return ok


def config_probe(rank, size):
    """The backend's own view of its configuration (C++ Config::describe) next to
    the Python mirror's (config.current) -- both read the same PDCC_* variables."""
    from pytorch_distributed_collective_communication_amd import config
    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    return be.describe(), config.current().__dict__


def _make_opt(name):
    import torch

    return (torch.optim.SGD, {"lr": 0.05, "momentum": 0.9}) if name == "sgd" else (torch.optim.AdamW, {"lr": 1e-2})


def zero_train(rank, size, optim="adam", steps=5, device="cpu", dtype="float32", resume=False,
               bucket_bytes=256 << 20, micro=1):
    """ZeRO-style sharded DP (parallel.zero.ShardedOptimizer) on the MLP; returns
    (final flat params, sharded state bytes, resumed params or None, buckets whose
    reduce-scatter started during backward in the last step). With resume=True the
    optimizer is checkpointed after 3 steps, 2 more steps run, and a fresh model +
    optimizer restored from the checkpoint must reproduce them. micro > 1: gradient
    accumulation over micro-batches (all but the last under no_sync())."""
    import torch

    from pytorch_distributed_collective_communication_amd.models import MLP, synthetic_batch
    from pytorch_distributed_collective_communication_amd.parallel.zero import ShardedOptimizer

    d = _dev(device)
    dt = getattr(torch, dtype)
    cls, kw = _make_opt(optim)
    x, y = synthetic_batch(64, device=d)
    shard = 64 // size
    xs, ys = x[rank * shard:(rank + 1) * shard].to(dt), y[rank * shard:(rank + 1) * shard].to(dt)

    def build():
        torch.manual_seed(100 + rank)  # different init per rank: the broadcast must fix it
        m = MLP().to(d, dt)
        return m, ShardedOptimizer(m.parameters(), cls, bucket_bytes=bucket_bytes, **kw)

    def run(model, opt, n):
        mb = shard // micro
        for _ in range(n):
            for k in range(micro):
                loss = torch.nn.functional.mse_loss(model(xs[k * mb:(k + 1) * mb]), ys[k * mb:(k + 1) * mb]) / micro
                if k < micro - 1:
                    with opt.no_sync():
                        loss.backward()
                else:
                    loss.backward()
            opt.step()
            opt.zero_grad()

    def flat(model):
        return torch.cat([p.detach().float().reshape(-1).cpu() for p in model.parameters()]).tolist()

    model, opt = build()
    if not resume:
        run(model, opt, steps)
        return flat(model), opt.sharded_state_bytes(), None, opt.overlapped
    run(model, opt, 3)
    ck = opt.state_dict()
    run(model, opt, 2)
    m2, o2 = build()
    o2.load_state_dict(ck)
    run(m2, o2, 2)
    return flat(model), opt.sharded_state_bytes(), flat(m2), opt.overlapped


def zero_reference(optim="adam", steps=5):
    """Single process, full batch, same optimizer: what sharded DP must reproduce."""
    import torch

    from pytorch_distributed_collective_communication_amd.models import MLP, synthetic_batch

    cls, kw = _make_opt(optim)
    torch.manual_seed(100)
    model = MLP()
    x, y = synthetic_batch(64)
    opt = cls(model.parameters(), **kw)
    for _ in range(steps):
        opt.zero_grad()
        torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


def device_id_probe(rank, size, path, device="cuda"):
    """init_process_group(device_id=...) connects eagerly (torch calls
    eagerConnectSingleDevice on backends that report splitting support); a subgroup
    that leaves the last rank out makes torch ask that rank for a no-color split
    (perform_nocolor_split, a no-op here). Re-initialises the world on a FileStore."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    dist.destroy_process_group()
    d = _dev(device)
    dist.init_process_group("mi355x", init_method="file://" + path, rank=rank, world_size=size, device_id=d)
    b = be.native_backend(None, "cuda")
    out = {"splitting": b.supports_splitting, "desc": b.describe(),
           "before": sorted(k for k in b.stats() if k.startswith("rccl_comm/"))}
    members = list(range(max(1, size - 1)))
    sub = dist.new_group(members)
    x = torch.full((4096,), float(rank + 1), device=d)
    dist.all_reduce(x)
    ok = bool(torch.all(x == size * (size + 1) / 2))
    if rank in members:
        y = torch.full((4096,), float(rank + 1), device=d)
        dist.all_reduce(y, group=sub)
        ok = ok and bool(torch.all(y == len(members) * (len(members) + 1) / 2))
    out["ok"] = ok
    return out


def object_collectives(rank, size, device="cpu"):
    """torch's pickled-object collectives (all_gather_object, broadcast_object_list,
    gather_object, scatter_object_list) run on top of our all_gather/broadcast/
    gather/scatter with variable-size uint8 payloads."""
    import torch.distributed as dist

    out = {}
    objs = [None] * size
    dist.all_gather_object(objs, {"r": rank, "s": "x" * (rank * 1000)})
    out["all_gather_object"] = [(o["r"], len(o["s"])) for o in objs]
    lst = [{"a": 1}, list(range(5000))] if rank == 0 else [None, None]
    dist.broadcast_object_list(lst, src=0)
    out["broadcast_object_list"] = [lst[0], len(lst[1])]
    g = [None] * size if rank == 0 else None
    dist.gather_object(("g", rank), g, dst=0)
    out["gather_object"] = g
    so = [None]
    dist.scatter_object_list(so, [("s", i) for i in range(size)] if rank == 0 else None, src=0)
    out["scatter_object_list"] = so[0]
    return out


def split_probe(rank, size, path, device="cuda"):
    """dist.split_group (ProcessGroup::splitGroup -> our Backend::split; torch needs
    the world bound to a device, so it is re-initialised with device_id on a
    FileStore): disjoint halves, an all_reduce and a broadcast inside each, then
    one on the world."""
    import torch
    import torch.distributed as dist

    dist.destroy_process_group()
    d = _dev(device)
    dist.init_process_group("mi355x", init_method="file://" + path, rank=rank, world_size=size, device_id=d)
    half = size // 2
    parts = [list(range(half)), list(range(half, size))]
    g = dist.split_group(split_ranks=parts)
    mine = parts[0] if rank < half else parts[1]
    x = torch.full((1000,), float(rank + 1), device=d)
    dist.all_reduce(x, group=g)
    y = torch.full((10,), float(rank), device=d)
    dist.broadcast(y, src=mine[0], group=g)
    z = torch.ones(3, device=d)
    dist.all_reduce(z)
    return {"sum": x[0].item(), "want": float(sum(r + 1 for r in mine)), "bcast": y[0].item(), "root": mine[0],
            "world": z[0].item(), "grank": dist.get_rank(g), "gsize": dist.get_world_size(g)}


def ll_probe(rank, size, device="cuda"):
    """LL all-reduce (<= 64 KiB): every dtype/op the kernels support, odd byte counts,
    many back-to-back calls (both slot parities, epoch rollover of the exit counter), a
    graph-captured sequence, in-place and out-of-place -- checked against exact sums."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    ok = {}
    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64, torch.uint8, torch.float64):
        for n in (1, 3, 7, 1000, 16383, (64 << 10) // torch.tensor([], dtype=dt).element_size()):
            x = (torch.arange(n, device=d) % 5 + rank + 1).to(dt)
            want = ((torch.arange(n, device=d) % 5) * size + size * (size + 1) // 2).to(dt)
            dist.all_reduce(x)
            ok[f"{dt}/{n}"] = bool(torch.equal(x, want))
    ok["algo"] = b.last_algo() == "ipc_ll"
    for opname in ("MAX", "MIN", "PRODUCT", "AVG"):
        x = torch.full((777,), float(rank + 1), device=d)
        dist.all_reduce(x, op=getattr(dist.ReduceOp, opname))
        want = {"MAX": size, "MIN": 1, "PRODUCT": float(torch.arange(1, size + 1).prod()),
                "AVG": (size + 1) / 2}[opname]
        ok[opname] = bool(torch.allclose(x, torch.full_like(x, want)))
    for dt in (torch.float32, torch.bfloat16, torch.uint8, torch.int64):  # LL all-gather: list and flat outputs
        for n in (1, 5, 999, (64 << 10) // torch.tensor([], dtype=dt).element_size()):
            src = (torch.arange(n, device=d) % 7 + rank).to(dt)
            outs = [torch.empty(n, dtype=dt, device=d) for _ in range(size)]
            dist.all_gather(outs, src)
            flat = torch.empty(n * size, dtype=dt, device=d)
            dist.all_gather_into_tensor(flat, src)
            want = [(torch.arange(n, device=d) % 7 + r).to(dt) for r in range(size)]
            ok[f"ag/{dt}/{n}"] = all(bool(torch.equal(o, w)) for o, w in zip(outs, want)) and bool(
                torch.equal(flat, torch.cat(want)))
    ok["ag_algo"] = b.last_algo() == "ipc_ll"
    y = torch.zeros(4096, device=d)
    for k in range(101):  # parities, and values that change every call
        y.fill_(float(rank + k))
        dist.all_reduce(y)
        if not torch.all(y == sum(r + k for r in range(size))):
            ok["loop"] = False
            break
    else:
        ok["loop"] = True
    from pytorch_distributed_collective_communication_amd.parallel.graphs import capture

    bufs = [torch.zeros(1000 * (i + 1), device=d) for i in range(4)]
    g = capture(lambda: [dist.all_reduce(t) for t in bufs], warmup=1)
    for it in range(3):
        for t in bufs:
            t.fill_(float(rank + it))
        g.replay()
        torch.cuda.synchronize()
        ok[f"graph{it}"] = all(bool(torch.all(t == sum(r + it for r in range(size)))) for t in bufs)
    return ok


def ll_rooted_probe(rank, size, device="cuda", iters=61):
    """Rooted LL collectives (reduce / broadcast / gather / scatter <= 64 KiB per rank): the
    reference's one-element demos, odd byte counts, every root, and a long interleaved run of
    all six kinds with the root moving every call (the token lines must keep every slot
    parity safe whatever the sequence), plus a graph-captured rooted sequence."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    ok, algos = {}, {}
    tri = size * (size + 1) / 2

    def run_all(n, root, k, dt=torch.float32):
        res = {}
        x = torch.full((n,), float(rank + 1 + k), device=d).to(dt)
        keep = x.clone()
        dist.reduce(x, dst=root)
        res["reduce"] = bool(torch.equal(x, torch.full_like(x, tri + size * k))) if rank == root else bool(
            torch.equal(x, keep))
        algos["reduce"] = b.last_algo()
        y = (torch.arange(n, device=d) % 9 + k).to(dt) if rank == root else torch.full((n,), -1.0, device=d).to(dt)
        dist.broadcast(y, src=root)
        res["broadcast"] = bool(torch.equal(y, (torch.arange(n, device=d) % 9 + k).to(dt)))
        algos["broadcast"] = b.last_algo()
        g_in = torch.full((n,), float(rank + k), device=d).to(dt)
        g_out = [torch.full((n,), -1.0, device=d).to(dt) for _ in range(size)] if rank == root else None
        dist.gather(g_in, gather_list=g_out, dst=root)
        if rank == root:
            res["gather"] = all(bool(torch.all(t == r + k)) for r, t in enumerate(g_out))
        algos["gather"] = b.last_algo()
        s_out = torch.full((n,), -1.0, device=d).to(dt)
        s_in = [torch.full((n,), float(10 * r + k), device=d).to(dt) for r in range(size)] if rank == root else None
        dist.scatter(s_out, scatter_list=s_in, src=root)
        res["scatter"] = bool(torch.all(s_out == 10 * rank + k))
        algos["scatter"] = b.last_algo()
        return res

    # the reference's demo sizes (main.py: one element) with every root, then odd and maximal sizes
    for root in range(size):
        for key, v in run_all(1, root, 0).items():
            ok[f"one/{root}/{key}"] = v
    for dt in (torch.float32, torch.bfloat16, torch.uint8):
        es = torch.tensor([], dtype=dt).element_size()
        for n in (3, 1001, (64 << 10) // es):
            for key, v in run_all(n, size - 1, 1, dt).items():
                ok[f"{dt}/{n}/{key}"] = v
    ok["algos"] = all(a == "ipc_ll" for a in algos.values()) or algos
    # interleaved: the root and the kind change every call, all-reduce / all-gather in between
    good = True
    for k in range(iters):
        root = (k * 7 + 3) % size
        good = all(run_all(1 + (k * 37) % 2000, root, k).values()) and good
        z = torch.full((513,), float(rank + k), device=d)
        dist.all_reduce(z)
        good = good and bool(torch.all(z == size * (size - 1) / 2 + size * k))
    ok["interleaved"] = good
    from pytorch_distributed_collective_communication_amd.parallel.graphs import capture

    bx = torch.zeros(700, device=d)
    rx = torch.zeros(300, device=d)

    def step():
        dist.broadcast(bx, src=size - 1)
        dist.reduce(rx, dst=0)

    g = capture(step, warmup=1)
    for it in range(3):
        bx.fill_(float(100 + it) if rank == size - 1 else -1.0)
        rx.fill_(float(rank + it))
        g.replay()
        torch.cuda.synchronize()
        ok[f"graph{it}"] = bool(torch.all(bx == 100 + it)) and (
            bool(torch.all(rx == size * (size - 1) / 2 + size * it)) if rank == 0 else bool(torch.all(rx == rank + it)))
    return ok


def ll_exchange_probe(rank, size, device="cuda", iters=41):
    """LL reduce_scatter / all_to_all (<= 64 KiB per chunk): list and flat forms, dtypes, odd
    sizes, ops, and a long run interleaved with the other LL kinds."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    ok, algos = {}, {}
    tri0 = size * (size - 1) / 2  # sum of ranks

    def rs_a2a(n, k, dt=torch.float32, op="SUM"):
        res = {}
        ins = [torch.full((n,), float(10 * rank + q + k), device=d).to(dt) for q in range(size)]
        o = torch.full((n,), -1.0, device=d).to(dt)
        dist.reduce_scatter(o, ins, op=getattr(dist.ReduceOp, op))
        vals = [10 * s + rank + k for s in range(size)]
        want = {"SUM": sum(vals), "MAX": max(vals), "MIN": min(vals)}[op]
        res["rs"] = bool(torch.all(o == want))
        algos["rs"] = b.last_algo()
        flat_out = torch.empty(n, device=d).to(dt)
        dist.reduce_scatter_tensor(flat_out, torch.cat(ins))
        res["rs_flat"] = bool(torch.all(flat_out == sum(vals)))
        outs = [torch.full((n,), -1.0, device=d).to(dt) for _ in range(size)]
        dist.all_to_all(outs, ins)
        res["a2a"] = all(bool(torch.all(t == 10 * q + rank + k)) for q, t in enumerate(outs))
        algos["a2a"] = b.last_algo()
        fo = torch.empty(n * size, device=d).to(dt)
        dist.all_to_all_single(fo, torch.cat(ins))
        res["a2a_flat"] = all(bool(torch.all(t == 10 * q + rank + k)) for q, t in enumerate(fo.view(size, n)))
        return res

    for dt in (torch.float32, torch.bfloat16, torch.int32):
        es = torch.tensor([], dtype=dt).element_size()
        for n in (1, 3, 1001, (64 << 10) // es):
            for key, v in rs_a2a(n, 0, dt).items():
                ok[f"{dt}/{n}/{key}"] = v
    for op in ("MAX", "MIN"):
        ok[f"op/{op}"] = rs_a2a(257, 1, op=op)["rs"]
    ok["algos"] = all(a == "ipc_ll" for a in algos.values()) or algos
    good = True
    for k in range(iters):
        good = all(rs_a2a(1 + (k * 53) % 3000, k).values()) and good
        z = torch.full((100,), float(rank + k), device=d)
        dist.broadcast(z, src=k % size)
        good = good and bool(torch.all(z == k % size + k))
        dist.all_reduce(z)
        good = good and bool(torch.all(z == size * (k % size + k)))
    ok["interleaved"] = good
    return ok


def partial_rows(rank, size, device="cuda", reps=6):
    """2-shot all-reduces whose last row of W tiles is partial (the padding tiles of that row
    are skipped by the pull pipeline), mixed with other sizes so every block's LDS ring holds
    stale tiles from earlier rows: every result must be exact, on the IPC 2-shot engine."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    ok, algos = {}, set()
    tri = size * (size + 1) / 2
    sizes = (1 << 20, 3 * size * 1024 + 257, (5 * size + size - 1) * 1024 + 100, (1 << 20) + 3 * 1024)
    for k in range(reps):
        for n in sizes:
            base = torch.arange(n, device=d).remainder(7).float()
            x = base + (rank + 1 + k)
            dist.all_reduce(x)
            algos.add(b.last_algo())
            key = f"{n}"
            ok[key] = ok.get(key, True) and bool(torch.equal(x, base * size + tri + size * k))
    ok["algos"] = all(a.startswith("ipc_2shot") for a in algos) or sorted(algos)
    return ok


def async_then_sync(rank, size, device="cuda", rounds=6):
    """An async collective still running on the group's comm stream, then a synchronous
    one on the caller's stream before wait(): the backend must order the second behind
    the first (same-group collectives never overlap), for every engine size class."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    ok = []
    for k in range(rounds):
        big = torch.full((4 << 20,), float(rank + k), device=d)      # 16 MiB: 2-shot / RCCL
        mid = torch.full((1 << 20,), float(rank + 2 * k), device=d)  # 4 MiB: 2-shot
        small = torch.full((1000,), float(rank + 3 * k), device=d)   # LL / 1-shot
        w = dist.all_reduce(big, async_op=True)
        dist.all_reduce(mid)
        dist.all_reduce(small)
        w.wait()
        tri = size * (size - 1) / 2
        ok.append(bool(torch.all(big == tri + size * k)) and bool(torch.all(mid == tri + 2 * size * k))
                  and bool(torch.all(small == tri + 3 * size * k)))
    return ok


def a2a_list_routing(rank, size, device="cuda"):
    """dist.all_to_all with tensor lists: equal chunks agree group-wide and take the IPC
    engines (LL <= 64 KiB, staged IPC at 1 MiB); one rank with an uneven chunk sends every
    rank to the generic path. Values checked in every case."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    res = {}
    for tag, n in (("ll", 1000), ("ipc", (1 << 20) // 4)):
        ins = [torch.full((n,), float(100 * rank + q), device=d) for q in range(size)]
        outs = [torch.full((n,), -1.0, device=d) for _ in range(size)]
        dist.all_to_all(outs, ins)
        res[tag] = (b.last_algo(), all(bool(torch.all(t == 100 * q + rank)) for q, t in enumerate(outs)))
    # uneven: rank 0 keeps a larger chunk for itself (its self-chunk only), everything else equal
    n = 1000
    sizes_in = [2 * n if (rank == 0 and q == 0) else n for q in range(size)]
    ins = [torch.full((sizes_in[q],), float(100 * rank + q), device=d) for q in range(size)]
    outs = [torch.full((2 * n if (rank == 0 and q == 0) else n,), -1.0, device=d) for q in range(size)]
    dist.all_to_all(outs, ins)
    res["uneven"] = (b.last_algo(), all(bool(torch.all(t == 100 * q + rank)) for q, t in enumerate(outs)))
    return res


def conformance_probe(rank, size, device="cuda", max_bytes=64 << 20):
    """The bench's conformance pass (utils/conformance.py) run as a test."""
    from pytorch_distributed_collective_communication_amd.utils import conformance

    return conformance.run(rank, size, _dev(device), deadline_s=120.0, max_bytes=max_bytes)


def zc_async_probe(rank, size, device="cuda", trials=5, n=16 << 20, late_ms=50):
    """Zero-copy calls exchange their buffer records on the launcher thread: rank 0's
    host must get an async 64 MiB all_reduce back at once while rank 1 is held back
    `late_ms`; a synchronous one as well (only the stream waits). Values checked."""
    import statistics

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    x = torch.full((n,), float(rank + 1), device=d)
    dist.all_reduce(x)  # first call: fresh export, mappings made and confirmed
    torch.cuda.synchronize()
    tri = size * (size + 1) / 2
    res = {"warm": bool(torch.all(x == tri)), "algo": b.last_algo()}
    for mode in ("async", "sync"):
        ret, ok = [], True
        for _ in range(trials):
            x.fill_(float(rank + 1))
            torch.cuda.synchronize()
            dist.barrier()
            if rank == 1:
                time.sleep(late_ms / 1e3)
            t0 = time.perf_counter()
            w = dist.all_reduce(x, async_op=(mode == "async"))
            ret.append((time.perf_counter() - t0) * 1e6)
            if w is not None:
                w.wait()
            torch.cuda.synchronize()
            ok = ok and bool(torch.all(x == tri))
        res[f"{mode}_ret_us"] = statistics.median(ret)
        res[f"{mode}_ok"] = ok
    res["desc"] = b.describe()
    return res


def zc_churn_probe(rank, size, device="cuda", allocs=40, n=(10 << 20) // 4 + 64):
    """More distinct allocations than the zero-copy cache holds (10 MiB each: every one
    its own caching-allocator segment): exports get evicted and their mappings closed
    once the last launch that read them is done (no device-wide sync: this probe itself
    only synchronises its stream, so a hipDeviceSynchronize in a trace would be the
    library's); every result right, the closing list drains at the barrier."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    bufs = [torch.full((n + 64 * i,), float(rank + i), device=d) for i in range(allocs)]
    ok = True
    for rnd in range(2):
        for i, t in enumerate(bufs):
            t.fill_(float(rank + i))
            w = dist.all_reduce(t, async_op=True)
            if i % 3 == 0:
                w.wait()
        torch.cuda.current_stream().synchronize()
        for i, t in enumerate(bufs):
            ok = ok and bool(torch.all(t == sum(r + i for r in range(size))))
    before = b.describe()
    churn = b.zc_counters()  # (resolved: every churn call's outcome is in)
    dist.barrier()  # releases what the launcher's thread queued (evicted mappings)
    x = torch.ones(n, device=d)
    dist.all_reduce(x)
    torch.cuda.current_stream().synchronize()
    algo = b.last_algo()
    last = b.zc_counters()
    return {"ok": ok and bool(torch.all(x == size)), "algo": algo, "desc": b.describe(), "before_barrier": before,
            "calls": 2 * allocs, "churn": churn, "last": last}


def zc_burst_probe(rank, size, device="cuda", calls=64, n=(4 << 20) // 4):
    """A burst of async zero-copy all_reduces (no wait()), then torch.cuda.synchronize(),
    then the tensors are refilled and reduced once more synchronously: every result exact
    (a kernel launched after the synchronize would corrupt the refilled data)."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    bufs = [torch.full((n,), float(rank + 1 + i % 3), device=d) for i in range(4)]
    for i in range(calls):
        dist.all_reduce(bufs[i % 4], async_op=True)
    torch.cuda.synchronize()
    ok = {}
    for i, b in enumerate(bufs):
        k = len(range(i, calls, 4))  # reductions this buffer got
        want = sum(r + 1 + i % 3 for r in range(size)) * size ** (k - 1)
        ok[f"burst{i}"] = bool(torch.all(b == want).item())
    for i, b in enumerate(bufs):
        b.fill_(float(rank + 1))
        dist.all_reduce(b)
    torch.cuda.synchronize()
    for i, b in enumerate(bufs):
        ok[f"after{i}"] = bool(torch.all(b == size * (size + 1) / 2).item())
    return ok


# elements per case: every size ragged (not a multiple of a 4 KiB tile or of W tiles)
_NUMERICS_SIZES = {"ll": (1, 777, 16381), "oneshot": (40_009, 100_003), "twoshot": (300_007, 1_000_003),
                   "zc": (700_001, 2_000_003), "push": (700_001, 2_000_003), "staged_algo": (700_001, 2_000_003),
                   "dyn": (700_001, 2_000_003, 9_000_011)}


def random_numerics(rank, size, device="cuda", mode="ll"):
    """Seeded random fp32 / bf16 / fp16 all_reduce (SUM / AVG / PRODUCT / MAX / MIN) and
    reduce_scatter (SUM) through ONE IPC protocol -- picked by the test's environment --
    against an fp64 torch reduction of every rank's input (each rank regenerates all of
    them; utils/conformance.py `_close`: MAX/MIN bitwise, SUM/AVG within (W+1) eps of
    sum|x|, PRODUCT within (W+1) eps of |prod|). Reference call sites: main.py:14-15,23-24.
    Returns {case: [ok, engine]}."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be
    from pytorch_distributed_collective_communication_amd.utils.conformance import _close, _seeded

    d = _dev(device)
    gb = be.native_backend(None, "cuda")
    out = {}
    dts = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16}
    for dtn, dt in dts.items():
        for n in _NUMERICS_SIZES[mode]:
            for k, op in enumerate(("SUM", "AVG", "PRODUCT", "MAX", "MIN")):
                lo, hi = (0.5, 1.5) if op == "PRODUCT" else (-1.0, 1.0)
                seed = 1000 * k + n % 997
                xs = [_seeded((n,), dt, seed + 31 * r, d, lo, hi) for r in range(size)]
                t = xs[rank].clone()
                dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
                out[f"all_reduce/{dtn}/{op}/{n}"] = [_close(t.cpu(), [x.cpu() for x in xs], op, size, dtn),
                                                     gb.last_algo()]
            # reduce_scatter of W ragged chunks (chunk sizes follow the same protocol thresholds / W)
            m = max(1, n // size)
            xs = [_seeded((size * m,), dt, 77 + n % 991 + 31 * r, d) for r in range(size)]
            o = torch.empty(m, dtype=dt, device=d)
            dist.reduce_scatter_tensor(o, xs[rank].clone())
            mine = [x[rank * m:(rank + 1) * m].cpu() for x in xs]
            out[f"reduce_scatter/{dtn}/SUM/{m}"] = [_close(o.cpu(), mine, "SUM", size, dtn), gb.last_algo()]
    dist.barrier()
    return out


def zx_steady_probe(rank, size, device="cuda", calls=100, n=(4 << 20) // 4):
    """Steady-state zero-copy: `calls` async all_reduces on one 4 MiB tensor. The buffer is
    mapped once; from then on the gated kernels resolve the peers' buffers on the device
    (zx_fast in describe() counts the launches that did, once their gate slots are reused)."""
    import re

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    x = torch.empty(n, device=d)
    ok = True
    for i in range(calls):
        x.fill_(float(rank + i))
        dist.all_reduce(x, async_op=True).wait()
        if i % 10 == 9:
            ok = ok and bool(torch.all(x == sum(r + i for r in range(size))))
    torch.cuda.current_stream().synchronize()
    desc = b.describe()
    m = re.search(r"zx_fast=(\d+), zx_host=(\d+)", desc)
    return {"ok": ok, "algo": b.last_algo(), "fast": int(m.group(1)) if m else -1,
            "host": int(m.group(2)) if m else -1, "desc": desc}


def rccl_init_deadline(rank, size, device="cuda"):
    """Rank 1 never builds its RCCL communicator (PDCC_TEST_RCCL_INIT_SKIP): rank 0's
    non-blocking creation must give up at PDCC_RCCL_INIT_TIMEOUT_S with a clear message,
    poison the group, and the group's next call must fail at once (reference: Gloo surfaces a
    dead peer in ~0.2 s; main.py:94 / main.py:11 build the communicators)."""
    import time

    import torch
    import torch.distributed as dist

    d = _dev(device)
    x = torch.ones(1 << 16, device=d)
    res = {}
    t0 = time.time()
    try:
        dist.all_reduce(x)
        torch.cuda.synchronize()
        res["first"] = "no error"
    except RuntimeError as e:
        res["first"] = str(e)[:400]
    res["first_s"] = time.time() - t0
    t1 = time.time()
    try:
        dist.all_reduce(x)
        res["second"] = "no error"
    except RuntimeError as e:
        res["second"] = str(e)[:400]
    res["second_s"] = time.time() - t1
    return res


def coalesced_probe(rank, size, device="cpu", n=64, base=4096, timing=False):
    """Coalesced collectives (verdict r3 Next #5): torch's _coalescing_manager fast path
    (all_reduce / all_gather_into_tensor / reduce_scatter_tensor) and dist.all_reduce_coalesced
    run as ONE collective per call, checked against fp64 references built from every rank's
    seeded members. Members are ragged (not multiples of 16 B), mixed-dtype for the all-gather,
    and one all_reduce member is a non-contiguous view. Returns {check: ok} plus the number of
    collectives the backend recorded per coalesced call (and, with timing, loop vs coalesced us)."""
    import time

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, d.type)
    sizes = [base + 13 * i + (i % 3) for i in range(n)] + [2 * base + 6]  # [n]: the strided member (even)

    def member(i, r, dt=torch.float32):
        g = torch.Generator().manual_seed(1000 * i + 17 * r)
        return (torch.rand(sizes[i], generator=g, dtype=torch.float64) - 0.5).to(dt)

    res = {}

    def colls():
        st = b.stats()
        return sum(v[0] for k, v in st.items() if not k.startswith(("coalesced/", "rccl_comm/")))

    # --- all_reduce through the coalescing manager (async), one strided member
    ts = [member(i, rank).to(d) for i in range(n)]
    strided = member(n, rank).to(d).view(2, -1).t()  # non-contiguous view of fresh storage
    c0 = colls()
    with dist._coalescing_manager(device=d, async_ops=True) as cm:
        for t in ts:
            dist.all_reduce(t)
        dist.all_reduce(strided)
    cm.wait()
    res["allreduce_collectives"] = colls() - c0
    ok = True
    for i, t in enumerate(ts + [strided]):
        want = sum(member(i, r).double() for r in range(size))
        got = t.cpu().double() if i < n else t.t().reshape(-1).cpu().double()
        ok = ok and torch.allclose(got, want, rtol=1e-5, atol=1e-6)
    res["allreduce_ok"] = bool(ok)
    # --- dist.all_reduce_coalesced with MAX (the older API, same backend entry point)
    ms = [member(i, rank).to(d) for i in range(8)]
    c0 = colls()
    dist.all_reduce_coalesced(ms, op=dist.ReduceOp.MAX)
    res["allreduce_coalesced_api_collectives"] = colls() - c0
    res["allreduce_coalesced_api_ok"] = all(
        torch.equal(m.cpu(), torch.stack([member(i, r) for r in range(size)]).max(0).values) for i, m in enumerate(ms))
    # --- all_gather_into_tensor, mixed dtypes
    dts = [torch.float32, torch.bfloat16, torch.int64, torch.float16]
    ins = [member(i, rank, dts[i % 4]).to(d) for i in range(n)]
    outs = [torch.empty(size * sizes[i], dtype=dts[i % 4], device=d) for i in range(n)]
    c0 = colls()
    with dist._coalescing_manager(device=d, async_ops=True) as cm:
        for o, x in zip(outs, ins):
            dist.all_gather_into_tensor(o, x)
    cm.wait()
    res["allgather_collectives"] = colls() - c0
    res["allgather_ok"] = all(torch.equal(outs[i].cpu(), torch.cat([member(i, r, dts[i % 4]) for r in range(size)]))
                              for i in range(n))
    # --- reduce_scatter_tensor, SUM
    rins = [torch.cat([member(i, 100 * rank + q) for q in range(size)]).to(d) for i in range(n)]
    routs = [torch.empty(sizes[i], device=d) for i in range(n)]
    c0 = colls()
    with dist._coalescing_manager(device=d, async_ops=True) as cm:
        for o, x in zip(routs, rins):
            dist.reduce_scatter_tensor(o, x)
    cm.wait()
    res["reduce_scatter_collectives"] = colls() - c0
    res["reduce_scatter_ok"] = all(
        torch.allclose(routs[i].cpu().double(), sum(member(i, 100 * r + rank).double() for r in range(size)),
                       rtol=1e-5, atol=1e-6) for i in range(n))
    if timing:  # 64 x 16 KiB all_reduce: per-member loop vs one coalesced call
        xs = [torch.rand(4096, device=d) for _ in range(n)]

        def loop():
            for x in xs:
                dist.all_reduce(x)

        def coal():
            with dist._coalescing_manager(device=d, async_ops=False):
                for x in xs:
                    dist.all_reduce(x)

        for name, fn in (("loop", loop), ("coalesced", coal)):
            fn()
            torch.cuda.synchronize()
            lat = []
            for _ in range(10):
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                lat.append(time.perf_counter() - t0)
            lat.sort()
            res[f"{name}_us"] = lat[len(lat) // 2] * 1e6
    dist.barrier()
    return res


def zc_churn_nobarrier_probe(rank, size, device="cuda", allocs=24, rounds=4, n=(10 << 20) // 4 + 64, sync=False):
    """async zero-copy all_reduces over more allocations than the export cache holds,
    with NO barrier anywhere (evicted mappings can only be closed at safe points): the list of
    evicted-but-open mappings must stay bounded (a full rank refuses fresh exports / imports, those
    calls run staged), every result exact, and a hot buffer reduced between them keeps running
    zero-copy and resolving on the device (zx_fast grows round after round)."""
    import re

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    bufs = [torch.full((n + 64 * i,), float(rank + i), device=d) for i in range(allocs)]
    hot = torch.empty(n, device=d)
    ok = True
    closing, fast, hot_algo = [], [], []

    def grab(key):
        m = re.search(key + r"=(\d+)", b.describe())
        return int(m.group(1)) if m else -1

    churn_algo = []
    for rnd in range(rounds):
        for i, t in enumerate(bufs):
            t.fill_(float(rank + i))
            if sync:  # synchronous calls, each finished on the host before the next (conformance's pattern)
                dist.all_reduce(t)
                torch.cuda.synchronize()
                churn_algo.append(b.last_algo())
            else:
                dist.all_reduce(t, async_op=True).wait()
            hot.fill_(float(rank + 1))
            dist.all_reduce(hot, async_op=True).wait()
            hot_algo.append(b.last_algo())
        torch.cuda.current_stream().synchronize()
        for i, t in enumerate(bufs):
            ok = ok and bool(torch.all(t == sum(r + i for r in range(size))))
        ok = ok and bool(torch.all(hot == size * (size + 1) / 2))
        closing.append(grab("zc_closing"))
        fast.append(grab("zx_fast"))
    return {"ok": ok, "closing": closing, "fast": fast, "refusals": grab("zc_full_refusals"),
            "hot_algo": sorted(set(hot_algo[allocs:])), "churn_algo": sorted(set(churn_algo)), "desc": b.describe()}

def async_grid_probe(rank, size, device="cuda", calls=6):
    """PDCC_IPC_ASYNC_GRID: async_op=True IPC launches run the capped grid (counted in
    describe(): async_capped), synchronous ones do not; every result exact."""
    import re

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    ok = True

    def capped():  # (0 before the group's IPC communicator exists)
        m = re.search(r"async_capped=(\d+)", b.describe())
        return int(m.group(1)) if m else 0

    res = {}
    for n in (1000, (4 << 20) // 4 + 7):  # LL and zero-copy 2-shot (+ staged rest)
        x = torch.empty(n, device=d)
        c0 = capped()
        for _ in range(calls):
            x.fill_(float(rank + 1))
            dist.all_reduce(x)
            ok = ok and bool(torch.all(x == size * (size + 1) / 2))
        res[f"sync_capped_{n}"] = capped() - c0
        c0 = capped()
        for _ in range(calls):
            x.fill_(float(rank + 1))
            dist.all_reduce(x, async_op=True).wait()
            ok = ok and bool(torch.all(x == size * (size + 1) / 2))
        res[f"async_capped_{n}"] = capped() - c0
    torch.cuda.synchronize()
    res["ok"] = ok
    return res


def coalesced_direct(rank, size, device="cpu"):
    """pdcc.distributed's direct coalesced entry points (one Python call, one collective)."""
    import torch

    import pytorch_distributed_collective_communication_amd.distributed as pdist

    d = _dev(device)
    ins = [torch.full((3 + i,), float(rank * 10 + i), device=d) for i in range(5)]
    outs = [torch.empty(size * (3 + i), device=d) for i in range(5)]
    pdist.all_gather_into_tensor_coalesced(outs, ins)
    ok_ag = all(torch.equal(outs[i].cpu(), torch.cat([torch.full((3 + i,), float(r * 10 + i)) for r in range(size)]))
                for i in range(5))
    rin = [torch.arange(size * (2 + i), dtype=torch.float32, device=d) + rank for i in range(5)]
    rout = [torch.empty(2 + i, device=d) for i in range(5)]
    w = pdist.reduce_scatter_tensor_coalesced(rout, rin, op=pdist.ReduceOp.MAX, async_op=True)
    w.wait()
    ok_rs = all(torch.equal(rout[i].cpu(), torch.arange(rank * (2 + i), (rank + 1) * (2 + i), dtype=torch.float32)
                            + (size - 1)) for i in range(5))
    return {"ag": ok_ag, "rs": ok_rs}


def phase_trace_probe(rank, size, device="cuda", calls=6, mib=8):
    """PDCC_IPC_TRACE: block 0's header stamps are ordered and every traced block of a
    2-shot all_reduce files its phase-1 and exit stamps into the same record."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    x = torch.empty((mib << 20) // 4, device=d)
    ok = True
    for _ in range(calls):
        x.fill_(float(rank + 1))
        dist.all_reduce(x)
        ok = ok and bool(torch.all(x == size * (size + 1) / 2))
    torch.cuda.synchronize()
    HDR, NB = 24, 256  # kern::kTraceWords, kern::kTraceBlocks
    recs = [r for r in b.ipc_trace() if r[1] and r[7]]
    out = {"ok": ok, "engine": b.last_algo(), "records": len(recs), "rec_words": len(recs[-1]) if recs else 0}
    if recs:
        r = recs[-1]
        out["header_ordered"] = r[1] <= r[2] <= r[4] <= r[5] <= r[6] <= r[7]
        ex = [v for v in r[HDR + NB:HDR + 2 * NB] if v >= r[1]]
        p1 = [v for v in r[HDR:HDR + NB] if v >= r[1]]
        out["blocks_exit"] = len(ex)
        out["blocks_phase1"] = len(p1)
        out["slowest_exit_after_block0_us"] = (max(ex) - r[7]) / 100.0 if ex else None
        out["phase1_before_exit"] = all(a <= e for a, e in zip(r[HDR:HDR + NB], r[HDR + NB:HDR + 2 * NB]) if a)
    return out


def dyn_stress(rank, size, device="cuda", calls=60):
    """The dynamic zero-copy all-reduce (PDCC_ALGO=ipc_dyn) over many calls: sizes from a few
    chunks to thousands, synchronous and async (with PDCC_IPC_ASYNC_GRID set: the capped grid,
    another chunk size), interleaved with LL all_reduces and a barrier. Position-dependent,
    integer-valued data (exact in fp32): a wrong row, chunk or peer index changes the result."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    W = size
    tri = W * (W + 1) / 2

    def pos(n):  # 0..1020 by position (no period aligned to a tile or chunk)
        return (torch.arange(n, device=d) % 1021).float()

    sizes = [(1 << 20) // 4, (8 << 20) // 4 + 3, (64 << 20) // 4, (3 << 20) // 4 + 1024]
    bufs = [torch.empty(n, device=d) for n in sizes]
    bases = [pos(n) for n in sizes]
    small = torch.empty(1000, device=d)
    m = (4 << 20) // 4
    ag_in = torch.empty(m, device=d)
    ag_out = torch.empty(size * m, device=d)
    rs_in = torch.empty(size * m, device=d)
    rs_out = torch.empty(m, device=d)
    base_m, base_rs = pos(m), pos(size * m)
    ok, engines = True, set()
    for i in range(calls):
        k = i % len(bufs)
        x, base = bufs[k], bases[k]
        torch.add(base * (rank + 1), float(i % 7), out=x)
        if i % 3 == 2:
            dist.all_reduce(x, async_op=True).wait()
        else:
            dist.all_reduce(x)
        engines.add(b.last_algo())
        ok = ok and bool(torch.equal(x, base * tri + W * (i % 7)))
        if i % 5 == 4:
            small.fill_(1.0)
            dist.all_reduce(small)
            ok = ok and bool(torch.all(small == size))
        if i % 4 == 1:  # the dynamic all-gather and reduce-scatter (4 MiB per rank)
            torch.add(base_m, float(1000 * rank + i), out=ag_in)
            dist.all_gather_into_tensor(ag_out, ag_in)
            engines.add(b.last_algo())
            want_ag = torch.cat([base_m + float(1000 * r + i) for r in range(size)])
            ok = ok and bool(torch.equal(ag_out, want_ag))
            torch.add(base_rs * (rank + 1), float(i % 3), out=rs_in)
            dist.reduce_scatter_tensor(rs_out, rs_in)
            engines.add(b.last_algo())
            want_rs = base_rs[rank * m:(rank + 1) * m] * tri + W * (i % 3)
            ok = ok and bool(torch.equal(rs_out, want_rs))
        if i % 11 == 10:
            dist.barrier()
    torch.cuda.synchronize()
    return {"ok": ok, "engines": sorted(engines), "desc": b.describe()}


def mixed_async_op(rank, size, device="cuda", expect_error=False):
    """Rank 0 issues every all_reduce / all_gather / reduce_scatter with async_op=True, the other
    ranks synchronously (torch treats async_op as rank-local). Position-dependent data; every
    result exact. `expect_error`: return the first error instead (PDCC_DEBUG with a cap set)."""
    import re

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    tri = size * (size + 1) / 2
    asy = rank == 0
    ok = True
    try:
        for n in (1000, (256 << 10) // 4 + 5, (4 << 20) // 4 + 7, (24 << 20) // 4):
            base = (torch.arange(n, device=d) % 1021).float()
            for _ in range(3):
                x = base * (rank + 1)
                w = dist.all_reduce(x, async_op=asy)
                if asy:
                    w.wait()
                ok = ok and bool(torch.equal(x, base * tri))
            m = max(1, n // size)
            ag_in = base[:m] + 1000.0 * rank
            ag_out = torch.empty(size * m, device=d)
            w = dist.all_gather_into_tensor(ag_out, ag_in, async_op=asy)
            if asy:
                w.wait()
            ok = ok and bool(torch.equal(ag_out, torch.cat([base[:m] + 1000.0 * r for r in range(size)])))
            rs_in = torch.cat([base[:m] * (rank + 1) + q for q in range(size)])
            rs_out = torch.empty(m, device=d)
            w = dist.reduce_scatter_tensor(rs_out, rs_in, async_op=asy)
            if asy:
                w.wait()
            ok = ok and bool(torch.equal(rs_out, base[:m] * tri + size * rank))
        torch.cuda.synchronize()
    except RuntimeError as e:
        if expect_error:
            return {"error": str(e)[:400]}
        raise
    m = re.search(r"async_capped=(\d+)", b.describe())
    return {"ok": ok, "capped": int(m.group(1)) if m else 0, "error": ""}


def zc_size_guard_probe(rank, size, device="cuda", mib=2050):
    """bf16 all_gather_into_tensor of a `mib`-MiB input per rank (its own allocation): a size with
    bit 31 set is refused by the zero-copy export (IpcComm::zc_export -- a peer's mapping of it
    stalls) and runs staged, so the call completes at once; plus a 64 MiB call that still maps."""
    import re
    import time

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    out = {}
    for tag, m in (("big", mib), ("small", 64)):
        per = (m << 20) // 2
        x = torch.full((per,), float(rank), dtype=torch.bfloat16, device=d)
        y = torch.zeros(per * size, dtype=torch.bfloat16, device=d)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(2):
            dist.all_gather_into_tensor(y, x)
        torch.cuda.synchronize()
        out[f"{tag}_s"] = time.perf_counter() - t0
        smp = y.view(size, per)[:, ::4096].float()
        want = torch.arange(size, dtype=torch.float32)
        out[f"{tag}_ok"] = torch.equal(smp.amax(1).cpu(), want) and torch.equal(smp.amin(1).cpu(), want)
        out[f"{tag}_engine"] = b.last_algo()
        del x, y
        torch.cuda.empty_cache()
        m2 = re.search(r"zc_size_refusals=(\d+)", b.describe())
        out[f"{tag}_refusals"] = int(m2.group(1)) if m2 else -1
    return out


def distinct_suite(rank, size, device, phases, store_dir):
    """One launch for many distinct-GPU checks (verdict r5 Next #6: the GPU suite's multi-GPU layer
    in one process set per world size instead of one per parametrization). `phases` =
    [(key, worker name, args, env)]: for each, the phase's environment is applied (the backend reads
    its PDCC_* configuration when a group is made), the default group is re-made on a FileStore of its
    own, and the worker runs; {key: result, or {"__error__": message}} per rank."""
    import datetime
    import os

    import torch.distributed as dist

    out = {}
    for k, (key, fname, args, env) in enumerate(phases):
        saved = {n: os.environ.get(n) for n in env}
        os.environ.update({n: str(v) for n, v in env.items()})
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
            store = dist.FileStore(os.path.join(store_dir, f"phase{k}"), size)
            dist.init_process_group("mi355x", store=store, rank=rank, world_size=size,
                                    timeout=datetime.timedelta(seconds=120))
            out[key] = globals()[fname](rank, size, *args)
        except Exception as e:  # noqa: BLE001 - recorded per phase; the test that owns it fails
            out[key] = {"__error__": f"{type(e).__name__}: {e}"[:800]}
        finally:
            for n, v in saved.items():
                if v is None:
                    os.environ.pop(n, None)
                else:
                    os.environ[n] = v
    return out


def size_guard_vote_probe(rank, size, device="cuda"):
    """rank 1 lifts the zero-copy size guard for a new group, rank 0 does not; the
    group's first GPU collective votes, and both ranks end with the guard on (a guarded rank must never
    import a record a rank without the guard exported)."""
    import os
    import re

    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    if rank == 1:
        os.environ["PDCC_IPC_ZC_SIZE_GUARD"] = "0"
    g = dist.new_group(list(range(size)))
    os.environ.pop("PDCC_IPC_ZC_SIZE_GUARD", None)
    b = be.native_backend(g, "cuda")
    before = re.search(r"ipc_zc_size_guard=(\d)", b.describe()).group(1)
    x = torch.ones(1 << 20, device=_dev(device))
    dist.all_reduce(x, group=g)
    torch.cuda.synchronize()
    after = re.search(r"ipc_zc_size_guard=(\d)", b.describe()).group(1)
    return {"before": before, "after": after, "ok": bool(torch.all(x == size))}


def bulk_diag(rank, size, device="cuda", n=3_000_017):
    """Diagnostics of the bulk all_reduce: engine, mismatch count, first bad index / value."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    base = torch.arange(n, dtype=torch.float32, device=d) % 1000
    t = base * (rank + 1)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    want = base * (size * (size + 1) // 2)
    bad = (t != want).nonzero().flatten()
    out = {"engine": be.native_backend(None, "cuda").last_algo(), "bad": int(bad.numel())}
    if bad.numel():
        i = int(bad[0])
        out.update(first=i, last=int(bad[-1]), got=float(t[i]), want=float(want[i]),
                   got_over_base=float(t[i] / base[i]) if float(base[i]) else None)
    out["zc"] = dict(be.native_backend(None, "cuda").zc_counters())
    return out


def ll_small(rank, size, device="cuda", calls=20, kind="all_reduce"):
    """`calls` small (LL-range) collectives of one kind, synchronised at the end."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    ok = True
    for i in range(calls):
        t = torch.full((1024,), float(rank + 1 + i), device=d)
        if kind == "all_reduce":
            dist.all_reduce(t)
            ok = ok and bool(torch.all(t == sum(r + 1 + i for r in range(size))))
        elif kind == "broadcast":
            dist.broadcast(t, src=0)
            ok = ok and bool(torch.all(t == 1 + i))
        elif kind == "reduce":
            dist.reduce(t, dst=0)
            ok = ok and (rank != 0 or bool(torch.all(t == sum(r + 1 + i for r in range(size)))))
    torch.cuda.synchronize()
    return ok


def canary(rank, size, device="cuda", n=16 << 20, wait_s=1.0):
    """Rogue-writer check: a fresh tensor filled with 7.0 must stay 7.0 while nothing runs."""
    import time

    import torch

    d = _dev(device)
    x = torch.full((n,), 7.0, device=d)
    torch.cuda.synchronize()
    time.sleep(wait_s)
    torch.cuda.synchronize()
    return int((x != 7.0).sum())


def regroup_probe(rank, size, device="cuda", destroy_a=True, b_first=False, n=3_000_017, b_algo=None, sleep_s=0.0,
                  repeat=1, warm=False):
    """Group A runs small (LL) all_reduces, then group B (same members) a bulk all_reduce. Per call:
    [mismatches of B's result, elements of `base` changed during the call, mismatches of the input
    before the call, first and last bad index]. `destroy_a`: A is destroyed before B's call;
    `b_first`: B is made before A runs anything; `warm`: B runs a 1-element all_reduce first."""
    import torch
    import torch.distributed as dist

    d = _dev(device)
    ranks = list(range(size))
    b = dist.new_group(ranks) if b_first else None
    a = dist.new_group(ranks)
    for i in range(5):
        t = torch.full((1024,), float(rank + 1), device=d)
        dist.all_reduce(t, group=a)
    torch.cuda.synchronize()
    if destroy_a:
        dist.destroy_process_group(a)
    if b is None:
        b = dist.new_group(ranks)
    if b_algo:
        from pytorch_distributed_collective_communication_amd.parallel import backend as be

        be.native_backend(b, "cuda").set_algo(b_algo)
    if sleep_s:
        import time

        time.sleep(sleep_s)
    if warm:
        w = torch.ones(1, device=d)
        dist.all_reduce(w, group=b)
    out = []
    for _ in range(repeat):
        base = torch.arange(n, dtype=torch.float32, device=d) % 1000
        t = base * (rank + 1)
        torch.cuda.synchronize()
        base_h = base.cpu()
        t_h = t.cpu()
        pre = int((t_h != base_h * (rank + 1)).sum())
        dist.all_reduce(t, group=b)
        torch.cuda.synchronize()
        bad = (t.cpu() != base_h * (size * (size + 1) // 2))
        nz = bad.nonzero()
        got = t.cpu()
        exp = base_h * (size * (size + 1) // 2)
        idx = nz.flatten()[:: max(1, len(nz) // 12)][:12].tolist()
        from pytorch_distributed_collective_communication_amd.parallel import backend as be

        out.append([int(bad.sum()), int((base.cpu() != base_h).sum()), pre,
                    int(nz[0]) if len(nz) else -1, int(nz[-1]) if len(nz) else -1,
                    [(i, float(got[i]), float(exp[i])) for i in idx], be.native_backend(b, "cuda").last_algo(),
                    hex(t.data_ptr()), hex(base.data_ptr()), os.getpid()])
    return out


def zc_reuse_diag(rank, size, device="cuda"):
    """The zero_copy worker's first steps with per-call diagnostics: the 4 all-reduces, then 10 fill +
    all_reduce calls on one 2 MiB buffer: [mismatches, engine] per call."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    tile = 1024
    tri = size * (size + 1) // 2
    out = []
    for n in (size * tile * 300, size * tile * 300 + 77, (1 << 20) // 4 + 3, 3 * size * tile * 256 + 1):
        base = torch.arange(n, device=d, dtype=torch.float32) % 1000
        t = base * (rank + 1)
        dist.all_reduce(t)
        out.append([int((t != base * tri).sum()), b.last_algo()])
    x = torch.empty(size * tile * 256, device=d)
    for _ in range(10):
        x.fill_(rank + 1.0)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        bad = (x != tri).nonzero().flatten()
        out.append([len(bad), b.last_algo(), bad[:4].tolist(), x[bad[:4]].tolist() if len(bad) else []])
    return {"calls": out[3:6], "zc": be.zc_counters(None), "x": hex(x.data_ptr()), "pid": os.getpid()}


def bulk_pre_diag(rank, size, device="cuda", n=3_000_017):
    """The default group's first bulk all_reduce: [result mismatches, input mismatches seen on the host
    before the call, engine, first bad index, (got, want) there]."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    base = torch.arange(n, dtype=torch.float32, device=d) % 1000
    t = base * (rank + 1)
    torch.cuda.synchronize()
    base_h = torch.arange(n, dtype=torch.float32) % 1000
    pre = int((t.cpu() != base_h * (rank + 1)).sum())
    dist.all_reduce(t)
    torch.cuda.synchronize()
    got = t.cpu()
    want = base_h * (size * (size + 1) // 2)
    bad = (got != want).nonzero().flatten()
    i = int(bad[0]) if len(bad) else -1
    return [len(bad), pre, be.native_backend(None, "cuda").last_algo(), i,
            (float(got[i]), float(want[i])) if i >= 0 else None]



def ll_unaligned_probe(rank, size, device="cuda"):
    """LL collectives on views of one flat tensor at 4-byte offsets (not 16-B / 8-B aligned), used in place
    (prep_in any_align, byte-wise LL lines): all_gather_into_tensor, reduce_scatter_tensor, all_to_all_single,
    scatter and gather through list views of one buffer, for 1, 3 and 1001 fp32 per rank -- exact against
    the expected values; plus the engine label."""
    import torch
    import torch.distributed as dist

    from pytorch_distributed_collective_communication_amd.parallel import backend as be

    d = _dev(device)
    b = be.native_backend(None, "cuda")
    ok, algos = {}, set()
    for n in (1, 3, 1001):
        src = torch.arange(n, device=d, dtype=torch.float32) + 1000 * rank
        flat = torch.full((n * size,), -1.0, device=d)
        dist.all_gather_into_tensor(flat, src)
        algos.add(b.last_algo())
        want = torch.cat([torch.arange(n, device=d, dtype=torch.float32) + 1000 * r for r in range(size)])
        ok[f"ag/{n}"] = bool(torch.equal(flat, want))
        # an offset input view too: element 1.. of a bigger buffer
        big = torch.zeros(n + 1, device=d)
        big[1:] = src
        flat2 = torch.full((n * size + 1,), -1.0, device=d)[1:]
        dist.all_gather_into_tensor(flat2, big[1:])
        ok[f"ag_offset/{n}"] = bool(torch.equal(flat2, want))
        inp = torch.arange(n * size, device=d, dtype=torch.float32) + rank
        out = torch.full((n,), -1.0, device=d)
        dist.reduce_scatter_tensor(out, inp)
        algos.add(b.last_algo())
        rs_want = (torch.arange(n * size, device=d, dtype=torch.float32) * size + size * (size - 1) / 2)[rank * n:(rank + 1) * n]
        ok[f"rs/{n}"] = bool(torch.equal(out, rs_want))
        a_in = torch.arange(n * size, device=d, dtype=torch.float32) + 100000 * rank
        a_out = torch.full((n * size,), -1.0, device=d)
        dist.all_to_all_single(a_out, a_in)
        algos.add(b.last_algo())
        a_want = torch.cat([torch.arange(rank * n, (rank + 1) * n, device=d, dtype=torch.float32) + 100000 * q
                            for q in range(size)])
        ok[f"a2a/{n}"] = bool(torch.equal(a_out, a_want))
        sbuf = torch.arange(n * size, device=d, dtype=torch.float32) + 7
        s_out = torch.full((n,), -1.0, device=d)
        dist.scatter(s_out, scatter_list=list(sbuf.split(n)) if rank == 0 else None, src=0)
        ok[f"scatter/{n}"] = bool(torch.equal(s_out, sbuf[rank * n:(rank + 1) * n]))
        gbuf = torch.full((n * size,), -1.0, device=d)
        dist.gather(src, gather_list=list(gbuf.split(n)) if rank == 0 else None, dst=0)
        if rank == 0:
            ok[f"gather/{n}"] = bool(torch.equal(gbuf, want))
        # in-place collectives on a view at a 4-byte offset: all_reduce, reduce, broadcast
        buf = torch.full((n + 1,), -5.0, device=d)
        v = buf[1:]
        v.copy_(torch.arange(n, device=d, dtype=torch.float32) + rank)
        dist.all_reduce(v)
        algos.add(b.last_algo())
        ar_want = torch.arange(n, device=d, dtype=torch.float32) * size + size * (size - 1) / 2
        ok[f"ar_offset/{n}"] = bool(torch.equal(v, ar_want)) and float(buf[0]) == -5.0
        v.copy_(torch.arange(n, device=d, dtype=torch.float32) + rank)
        dist.reduce(v, dst=0)
        if rank == 0:
            ok[f"reduce_offset/{n}"] = bool(torch.equal(v, ar_want)) and float(buf[0]) == -5.0
        v.copy_(torch.arange(n, device=d, dtype=torch.float32) * (3 if rank == 0 else 0))
        dist.broadcast(v, src=0)
        ok[f"bcast_offset/{n}"] = bool(torch.equal(v, torch.arange(n, device=d, dtype=torch.float32) * 3)) and \
            float(buf[0]) == -5.0
    return {"ok": ok, "algos": sorted(algos)}
