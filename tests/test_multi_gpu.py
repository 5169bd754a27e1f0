"""One rank per distinct MI355X (RCCL over xGMI and the IPC peer-memory path
across devices). Runs only where torch sees at least `world` GPUs; on the
1-GPU box these skip with a reason (the driver's multi-GPU node runs them).

Each data path is forced in turn (PDCC_ALGO=rccl / ipc / ...) and left to the
autotuner (auto), against the reference's golden outputs (README.md:105-284,
SURVEY.md §4.2) and, for random data, RCCL against IPC on the same inputs.

Budget (verdict r5 Next #6): every check of one world size runs in ONE launch
(tests/_workers.py ``distinct_suite``: per phase the environment is applied and
the default group re-made on its own FileStore), so the layer costs four
process starts -- W = 2, 3, 4, 8 -- instead of one per parametrization. The
tests below read their phase's per-rank results from that launch; estimate in
profiles/r6/gpu_suite_budget.md.
"""
import functools
import tempfile

import pytest
import torch

from pytorch_distributed_collective_communication_amd.parallel.spawn import launch
from tests import _workers as W

pytestmark = pytest.mark.gpu

_ZC_ENV = {"PDCC_IPC_ZC_CACHE": "4", "PDCC_IPC_1SHOT_MAX": "256K", "PDCC_IPC_MAX_STAGING": "8M"}
_TUNED = ("rccl", "rccl_wide", "ipc", "ipc_wide", "ipc_push", "ipc_staged", "ipc_dyn", "ipc_sdma")


def _plan(world, store_dir):
    """(key, worker, args, env) phases of one world size, in run order."""
    c = "cuda"
    p = []
    if world in (2, 4, 8):
        p += [(f"golden/{a}", "golden", (c,), {"PDCC_ALGO": a}) for a in ("rccl", "ipc", "auto")]
        p += [("conformance", "conformance_probe", (c,), {})]
        p += [(f"zero_copy/{a}", "zero_copy", (c,), {"PDCC_ALGO": a, **_ZC_ENV}) for a in ("ipc", "ipc_push", "ipc_wide")]
        p += [("ll", "ll_probe", (c,), {"PDCC_ALGO": "ipc"}), ("ll_rooted", "ll_rooted_probe", (c,), {"PDCC_ALGO": "ipc"}),
              ("ll_exchange", "ll_exchange_probe", (c,), {"PDCC_ALGO": "ipc"})]
    if world in (2, 3, 8):
        p += [(f"bulk/{a}", "large", (c,), {"PDCC_ALGO": a}) for a in ("rccl", "ipc", "auto")]
    if world == 2:
        p += [(f"autotune/{n}", "autotune_all_colls", (c, n), {"PDCC_IPC_LL_MAX": "64K"}) for n in (1 << 16, 1 << 22)]
        p += [(f"group_churn/{m}", "group_churn", (c,), {"PDCC_RCCL_GROUP_COMM": m}) for m in ("share", "split")]
        p += [(f"graph/{a}", "graph_capture", (c,), {"PDCC_ALGO": a} if a else {}) for a in ("rccl", "ipc", "")]
        p += [("async_ordering", "async_ordering", (c,), {"PDCC_STREAM": "comm"})]
        p += [(f"sync_after_async/{a}", "async_then_sync", (c,), {"PDCC_ALGO": a}) for a in ("rccl", "ipc", "auto")]
    if world in (2, 4):
        p += [("zero_train", "zero_train", ("adam", 5, c, "float32", False, 4096), {}),
              ("device_id", "device_id_probe", (f"{store_dir}/device_id",), {})]
    if world == 4:
        p += [(f"op_matrix/{a}", "op_matrix", (c, ("float32", "int32", "bfloat16", "int64")), {"PDCC_ALGO": a})
              for a in ("rccl", "ipc")]
        p += [(f"list_all_gather/{g}", "large", (c,), {"PDCC_ALGO": "rccl", "PDCC_LIST_GATHER": g})
              for g in ("p2p", "staged")]
        p += [("crosscheck", "engine_crosscheck", (c,), {}), ("p2p", "p2p_subset", (c, 1 << 18), {}),
              ("split", "split_probe", (f"{store_dir}/split",), {})]
    return p


@functools.lru_cache(maxsize=None)
def _suite(world):
    store_dir = tempfile.mkdtemp(prefix=f"pdcc_distinct_w{world}_")
    return launch(W.distinct_suite, world, args=("cuda", tuple(_plan(world, store_dir)), store_dir),
                  bind_device=True, timeout_s=120, join_timeout_s=1500)


def _phase(world, key):
    n = torch.cuda.device_count()
    if n < world:
        pytest.skip(f"needs {world} GPUs (one rank per device), {n} visible")
    res = [r[key] for r in _suite(world)]
    errs = [r["__error__"] for r in res if isinstance(r, dict) and "__error__" in r]
    assert not errs, errs
    return res


def test_plan_covers_every_world():
    # (no GPU: the phase lists themselves) each world size has its checks, keys are unique
    for w in (2, 3, 4, 8):
        keys = [k for k, *_ in _plan(w, "/tmp/x")]
        assert keys and len(keys) == len(set(keys)), (w, keys)


@pytest.mark.parametrize("algo", ["rccl", "ipc", "auto"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_golden_distinct_gpus(world, algo):
    for r, got in enumerate(_phase(world, f"golden/{algo}")):
        assert got == W.expected_golden(r, world), (r, got)


@pytest.mark.parametrize("algo", ["rccl", "ipc"])
def test_op_matrix_distinct_gpus(algo):
    world = 4
    for got in _phase(world, f"op_matrix/{algo}"):
        for key, val in got.items():
            kind, dt, op = key.split("/")
            exp = W.expected_op(world, op)
            assert val == (pytest.approx(exp, rel=1e-2) if dt == "bfloat16" else pytest.approx(exp)), key


@pytest.mark.parametrize("algo", ["rccl", "ipc", "auto"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_bulk_and_lists_distinct_gpus(world, algo):
    for ok in _phase(world, f"bulk/{algo}"):
        assert all(ok.values()), ok


@pytest.mark.parametrize("gather", ["p2p", "staged"])
def test_list_all_gather_engines(gather):
    for ok in _phase(4, f"list_all_gather/{gather}"):
        assert all(ok.values()), ok


def test_rccl_and_ipc_agree_on_random_data():
    for ok in _phase(4, "crosscheck"):
        assert all(ok.values()), ok


@pytest.mark.parametrize("n", [1 << 16, 1 << 22])
def test_autotuner_distinct_gpus(n):
    # 256 KiB keys (tuned, not LL) and 16 MiB keys (verdict r4 weak #3: the bulk race the 1 GiB
    # headline runs -- zero-copy, staged, push, dynamic, wide and copy-engine candidates -- on distinct devices)
    res = _phase(2, f"autotune/{n}")
    for r in res:
        assert all(r["ok"].values()), r["ok"]
    assert res[0]["table"] == res[1]["table"]
    for e in res[0]["table"]:
        assert e["ipc_valid"], e
        if e["op"] in ("BAND", "BOR"):  # no RCCL op: the host transport is the reference engine
            assert e["ref"] == "host" and e["algo"] in ("host",) + _TUNED, e
        else:
            assert e["ref"] == "rccl" and e["algo"] in _TUNED, e
    if n >= 1 << 20:
        ar = [e for e in res[0]["table"] if e["coll"] == "allreduce" and e["op"] == "SUM" and e["lo"] >= 1 << 20]
        assert ar and all(e["dyn_us"] > 0 and e["staged_us"] > 0 and e["push_us"] > 0 for e in ar), ar


@pytest.mark.parametrize("world", [2, 4, 8])
def test_conformance_pass_distinct_gpus(world):
    # the bench's conformance pass (the driver's only distinct-GPU correctness gate), with every
    # engine the autotuner can adopt forced, the coalesced collectives, the async capped grid, the
    # raced bulk keys (verdict r4 Next #1), the ReduceOps at zero-copy / bulk sizes on every engine
    # and the copy-engine engine (verdict r5 Next #2 / #4)
    for r in _phase(world, "conformance"):
        assert r["all_ok"], {k: v for k, v in r["checks"].items() if not v["ok"]}
        names = set(r["checks"])
        for want in ("dyn/all_gather", "dyn/reduce_scatter", "staged/all_reduce", "wide/all_reduce",
                     "rccl_wide/all_reduce", "coalesced/ipc/all_reduce_x64", "coalesced/rccl/reduce_scatter_x64",
                     "async_capped/ipc/all_reduce", "raced/all_reduce/float32/SUM/24MiB",
                     "raced/all_reduce/int32/BXOR/24MiB", "ops/rccl/all_reduce/PRODUCT/64MiB",
                     "ops/rccl/reduce/SUM/64MiB_nonroot_untouched", "ops/ipc_push/all_reduce/MIN/64MiB",
                     "sdma/all_gather", "sdma/broadcast", "sdma/all_to_all"):
            assert want in names, (want, sorted(names))


@pytest.mark.parametrize("mode", ["share", "split"])
def test_group_churn_distinct_gpus(mode):
    for r in _phase(2, f"group_churn/{mode}"):
        assert all(r["ok"]), r
        for g in r["groups"]:
            assert g["how"] == [mode], r


@pytest.mark.parametrize("algo", ["rccl", "ipc", ""])
def test_graph_capture_distinct_gpus(algo):
    for ok in _phase(2, f"graph/{algo}"):
        assert all(ok), ok


def test_p2p_pairs_distinct_gpus():
    # send/recv between two ranks of a 4-rank group before any collective (2-rank
    # RCCL communicators), then a ring of first isends on a new group
    for ok in _phase(4, "p2p"):
        assert all(ok.values()), ok


def test_async_ordering_distinct_gpus():
    for ok in _phase(2, "async_ordering"):
        assert all(ok), ok


@pytest.mark.parametrize("algo", ["ipc", "ipc_push", "ipc_wide"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_zero_copy_distinct_gpus(world, algo):
    # peers read (ipc) / write (ipc_push) each other's tensors over xGMI; a small export
    # cache forces evictions, a small staging cap forces chunked push / rooted-reduce calls
    for ok in _phase(world, f"zero_copy/{algo}"):
        assert all(ok.values()), ok


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_optimizer_distinct_gpus(world):
    # ZeRO-style step: bucket reduce-scatters (AVG) launched during backward, all-gather of params
    res = _phase(world, "zero_train")
    ref = W.zero_reference("adam")
    for params, _, _, overlapped in res:
        assert params == res[0][0] and overlapped >= 2
        torch.testing.assert_close(torch.tensor(params), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("world", [2, 4])
def test_init_with_device_id_distinct_gpus(world):
    # eager RCCL communicator at init_process_group(device_id=...); the last rank is a
    # non-member of a subgroup (torch asks it for a no-color split)
    for r in _phase(world, "device_id"):
        assert r["ok"] and r["before"] == ["rccl_comm/init"], r


def test_split_group_distinct_gpus():
    # dist.split_group -> Backend::split: halves of a 4-GPU world, RCCL / IPC inside each
    for r, got in enumerate(_phase(4, "split")):
        assert got["sum"] == got["want"] and got["bcast"] == got["root"] and got["world"] == 4.0, got
        assert got["grank"] == r % 2 and got["gsize"] == 2, got


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ll_all_reduce_distinct_gpus(world):
    for ok in _phase(world, "ll"):
        assert all(ok.values()), ok


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ll_rooted_distinct_gpus(world):
    # reduce / broadcast / gather / scatter LL kernels over xGMI: data one way, tokens on the other pairs
    for ok in _phase(world, "ll_rooted"):
        ok = dict(ok)
        assert ok.pop("algos") is True, ok
        assert all(ok.values()), ok


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ll_reduce_scatter_all_to_all_distinct_gpus(world):
    for ok in _phase(world, "ll_exchange"):
        ok = dict(ok)
        algos = ok.pop("algos")
        assert algos is True or algos.get("rs") == "ipc_ll", algos
        assert all(ok.values()), ok


@pytest.mark.parametrize("algo", ["rccl", "ipc", "auto"])
def test_sync_collective_after_async_distinct_gpus(algo):
    for ok in _phase(2, f"sync_after_async/{algo}"):
        assert all(ok), ok
