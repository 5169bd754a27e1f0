#!/usr/bin/env python3
"""nccl-tests-style benchmark of the six collectives.

    python benchmarks/coll_bench.py --world 4 --backend mi355x --device cpu \
        --colls all_reduce,broadcast --sizes 4,1M,1G --iters 5
    # GPUs (one process per GPU):
    python benchmarks/coll_bench.py --world 8 --device cuda --sizes 1G

Method (same as BASELINE.md §2): spawn ``world`` processes, ``init_process_group``
then ``new_group(range(world))`` exactly like the reference (main.py:11,94);
per iteration ``barrier`` + timed collective; p50 = median over iterations of the
max-over-ranks time. busbw factors: all_reduce 2(n-1)/n; reduce and broadcast 1;
gather, scatter, all_gather, reduce_scatter, all_to_all (n-1)/n on the total
bytes. Inputs are reset before every timed call (outside the clock) and the
results of every timed bulk call are checked against independently computed
values (correctness is part of the benchmark). Prints one JSON line per (collective, op, dtype, size).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

COLLS = ["all_reduce", "reduce", "broadcast", "all_gather", "gather", "scatter", "reduce_scatter", "all_to_all"]


def parse_size(s: str) -> int:
    s = s.strip()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    if s[-1].upper() in mult:
        return int(float(s[:-1]) * mult[s[-1].upper()])
    return int(s)


def busbw_factor(coll: str, n: int) -> float:
    if n <= 1:
        return 0.0
    if coll == "all_reduce":
        return 2 * (n - 1) / n
    if coll in ("reduce", "broadcast"):
        return 1.0
    return (n - 1) / n


def worker(rank, size, cfg):
    import torch
    import torch.distributed as dist

    dev = torch.device("cpu") if cfg["device"] == "cpu" else torch.device("cuda", torch.cuda.current_device())
    if cfg["device"] == "cpu":
        torch.set_num_threads(1)
    g = dist.new_group(list(range(size)))
    dtype = getattr(torch, cfg["dtype"])
    esz = torch.tensor([], dtype=dtype).element_size()
    rows = []

    def sync():
        dist.barrier(group=g)
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def max_t(v):
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
        return t.item()

    for coll in cfg["colls"]:
        for op_name in cfg["ops"] if coll in ("all_reduce", "reduce", "reduce_scatter") else ["-"]:
            op = getattr(dist.ReduceOp, op_name) if op_name != "-" else None
            for nbytes in cfg["sizes"]:
                # S = per-rank tensor bytes for all_reduce/reduce/broadcast; total bytes otherwise
                if coll in ("all_reduce", "reduce", "broadcast"):
                    n = max(1, nbytes // esz)
                    total = n * esz
                else:
                    n = max(1, nbytes // esz // size)
                    total = n * esz * size
                v = (torch.arange(n, device=dev) % 7 + 1).to(dtype)  # small integers: exact in every dtype
                x = v + rank
                reset = lambda: None  # noqa: E731
                if coll == "all_gather":
                    outs = [torch.empty(n, dtype=dtype, device=dev) for _ in range(size)]
                    fn = lambda: dist.all_gather(outs, x, group=g)  # noqa: E731
                elif coll == "gather":
                    outs = [torch.empty(n, dtype=dtype, device=dev) for _ in range(size)] if rank == 0 else []
                    fn = lambda: dist.gather(x, gather_list=outs if rank == 0 else None, dst=0, group=g)  # noqa: E731
                elif coll == "scatter":
                    ins = [v + q for q in range(size)] if rank == 0 else None
                    out = torch.empty(n, dtype=dtype, device=dev)
                    fn = lambda: dist.scatter(out, scatter_list=ins, src=0, group=g)  # noqa: E731
                elif coll == "reduce_scatter":
                    inp = torch.cat([v + rank + q for q in range(size)])
                    out = torch.empty(n, dtype=dtype, device=dev)
                    fn = lambda: dist.reduce_scatter_tensor(out, inp, op=op, group=g)  # noqa: E731
                elif coll == "all_to_all":
                    inp = torch.cat([v + 10 * rank + q for q in range(size)])
                    out = torch.empty(n * size, dtype=dtype, device=dev)
                    fn = lambda: dist.all_to_all_single(out, inp, group=g)  # noqa: E731
                elif coll in ("all_reduce", "reduce"):
                    buf = x.clone()
                    reset = lambda: buf.copy_(x)  # noqa: E731  (in place: every timed call starts from x)
                    if coll == "all_reduce":
                        fn = lambda: dist.all_reduce(buf, op=op, group=g)  # noqa: E731
                    else:
                        fn = lambda: dist.reduce(buf, dst=0, op=op, group=g)  # noqa: E731
                else:
                    buf = x.clone()
                    reset = lambda: buf.copy_(v if rank == 0 else torch.zeros_like(v))  # noqa: E731
                    fn = lambda: dist.broadcast(buf, src=0, group=g)  # noqa: E731
                for _ in range(cfg["warmup"]):
                    reset()
                    fn()
                lat = []
                oks = []
                iters = cfg["iters"] if nbytes >= (1 << 20) else max(cfg["iters"], cfg["small_iters"])
                for _ in range(iters):
                    reset()
                    sync()
                    t0 = time.perf_counter()
                    fn()
                    if dev.type == "cuda":
                        torch.cuda.synchronize()
                    lat.append(max_t(time.perf_counter() - t0))
                    if not oks or nbytes >= (1 << 20):  # check the result of every timed bulk call
                        oks.append(_check(coll, op_name, rank, size, v, locals(), torch))
                p50 = statistics.median(lat)
                rows.append({
                    "coll": coll, "op": op_name, "dtype": cfg["dtype"], "bytes": total, "world": size,
                    "p50_us": round(p50 * 1e6, 2), "algbw_GBps": round(total / p50 / 1e9, 3) if p50 > 0 else None,
                    "busbw_GBps": round(total * busbw_factor(coll, size) / p50 / 1e9, 3) if p50 > 0 else None,
                    "correct": all(oks),
                })
                del x, v
    return rows


def _reduce_ref(op_name, parts, torch):
    """Exact reduction of the per-rank inputs, in float64 on the host."""
    st = torch.stack([p.double().cpu() for p in parts])
    if op_name in ("SUM",):
        return st.sum(0)
    if op_name == "AVG":
        return st.mean(0)
    if op_name == "PRODUCT":
        return st.prod(0)
    if op_name == "MAX":
        return st.max(0).values
    if op_name == "MIN":
        return st.min(0).values
    raise ValueError(op_name)


def _close(got, ref, torch):
    g = got.double().cpu()
    exact = got.dtype in (torch.float64, torch.int32, torch.int64, torch.int8, torch.uint8)
    if exact or bool((ref.abs() < 256).all()):
        return bool(torch.equal(g, ref.to(got.dtype).double()))
    rtol = 1e-6 if got.dtype == torch.float32 else 1e-2
    return bool(torch.allclose(g, ref.to(got.dtype).double(), rtol=rtol, atol=0))


def _check(coll, op_name, rank, size, v, loc, torch):
    """Verify a result against values computed independently (inputs are rank-dependent
    small integers, so every engine's result is exact or within a rounding tolerance)."""
    try:
        if coll == "broadcast":
            return bool(torch.equal(loc["buf"], v))
        if coll == "all_gather":
            return all(bool(torch.equal(o, v + q)) for q, o in enumerate(loc["outs"]))
        if coll == "gather":
            return rank != 0 or all(bool(torch.equal(o, v + q)) for q, o in enumerate(loc["outs"]))
        if coll == "scatter":
            return bool(torch.equal(loc["out"], v + rank))
        if coll == "all_to_all":
            exp = torch.cat([v + 10 * q + rank for q in range(size)])
            return bool(torch.equal(loc["out"], exp))
        if coll == "reduce_scatter":
            return _close(loc["out"], _reduce_ref(op_name, [v + r + rank for r in range(size)], torch), torch)
        if coll == "all_reduce" or (coll == "reduce" and rank == 0):
            return _close(loc["buf"], _reduce_ref(op_name, [v + r for r in range(size)], torch), torch)
        if coll == "reduce":
            return True  # non-root buffers are unspecified
        return False
    except Exception:
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--backend", default="mi355x")
    ap.add_argument("--device", default="cpu", choices=["cpu", "cuda"])
    ap.add_argument("--colls", default=",".join(COLLS))
    ap.add_argument("--ops", default="SUM")
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--sizes", default="4,1M,64M")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--small-iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    cfg = dict(device=a.device, colls=a.colls.split(","), ops=a.ops.split(","), dtype=a.dtype,
               sizes=[parse_size(s) for s in a.sizes.split(",")], iters=a.iters, small_iters=a.small_iters,
               warmup=a.warmup)
    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch

    rows = launch(worker, a.world, args=(cfg,), backend=a.backend, bind_device=a.device == "cuda",
                  join_timeout_s=3600)[0]
    for r in rows:
        r["backend"] = a.backend
        r["device"] = a.device
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
