"""benchmarks/coll_bench.py checks what it measures: every collective x every
ReduceOp at world 3 on the host transport, rank-dependent inputs reset before
each timed call, every row must report correct=true (verdict r1: the reductions
used to be reported correct without a check)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_coll_bench_checks_every_collective_and_op():
    cmd = [sys.executable, os.path.join(ROOT, "benchmarks", "coll_bench.py"), "--world", "3", "--device", "cpu",
           "--ops", "SUM,PRODUCT,MAX,MIN", "--sizes", "4,64K,2M", "--iters", "2", "--small-iters", "2",
           "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    colls = {x["coll"] for x in rows}
    assert colls == {"all_reduce", "reduce", "broadcast", "all_gather", "gather", "scatter", "reduce_scatter",
                     "all_to_all"}
    assert {x["op"] for x in rows if x["coll"] == "all_reduce"} == {"SUM", "PRODUCT", "MAX", "MIN"}
    bad = [x for x in rows if not x["correct"]]
    assert not bad, bad


def test_coll_bench_bf16_sums_are_checked():
    cmd = [sys.executable, os.path.join(ROOT, "benchmarks", "coll_bench.py"), "--world", "2", "--device", "cpu",
           "--colls", "all_reduce,reduce_scatter", "--ops", "SUM,PRODUCT", "--dtype", "bfloat16", "--sizes", "1M",
           "--iters", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(rows) == 4 and all(x["correct"] for x in rows), rows
