"""Single-process unit tests: config mirror, busbw math, kernel references,
package wiring (no GPU, no subprocesses except where noted)."""
import os

import pytest
import torch

from pytorch_distributed_collective_communication_amd import config, ops, utils
from pytorch_distributed_collective_communication_amd.parallel.spawn import launch
from tests import _workers as W


def test_parse_bytes():
    assert config.parse_bytes("512K") == 512 << 10
    assert config.parse_bytes("8M") == 8 << 20
    assert config.parse_bytes("1GiB") == 1 << 30
    assert config.parse_bytes("4096") == 4096


def test_config_rccl_cta_knobs():
    from pytorch_distributed_collective_communication_amd import config

    c = config.current({"PDCC_RCCL_MIN_CTAS": "8", "PDCC_RCCL_MAX_CTAS": "32"})
    assert (c.rccl_min_ctas, c.rccl_max_ctas) == (8, 32)
    assert config.current({}).rccl_min_ctas == -1
    assert config.env_for(rccl_max_ctas=14) == {"PDCC_RCCL_MAX_CTAS": "14"}


def test_config_current_and_env_for():
    env = {"PDCC_ALGO": "ipc", "PDCC_IPC_2SHOT_MAX": "16M", "PDCC_DEBUG": "1", "PDCC_IPC": "0"}
    c = config.current(env)
    assert c.algo == "ipc" and c.ipc_2shot_max == 16 << 20 and c.debug and not c.ipc
    assert config.env_for(algo="rccl", debug=True) == {"PDCC_ALGO": "rccl", "PDCC_DEBUG": "1"}
    with pytest.raises(ValueError):
        config.current({"PDCC_ALGO": "bogus"})
    with pytest.raises(KeyError):
        config.env_for(nope=1)


def test_busbw_conventions():
    assert utils.busbw_factor("all_reduce", 8) == pytest.approx(1.75)
    assert utils.busbw_factor("broadcast", 8) == 1.0
    assert utils.busbw_factor("all_gather", 4) == pytest.approx(0.75)
    assert utils.busbw_factor("all_reduce", 1) == 0.0
    assert utils.busbw("all_reduce", 1 << 30, 2, 1.0) == pytest.approx((1 << 30) / 1e9)
    assert utils.xgmi_ceiling_GBps(8) == pytest.approx(7 * 153.0)
    assert utils.xgmi_ceiling_GBps(2) == pytest.approx(153.0)


@pytest.mark.parametrize("op", ["sum", "prod", "min", "max", "avg"])
def test_reduce_reference_float(op):
    xs = [torch.tensor([1.0, -2.0, 3.5]), torch.tensor([2.0, 4.0, -1.0]), torch.tensor([0.5, 1.0, 2.0])]
    got = ops.reduce_nway_reference(xs, op)
    exp = {"sum": xs[0] + xs[1] + xs[2], "prod": xs[0] * xs[1] * xs[2],
           "min": torch.minimum(torch.minimum(xs[0], xs[1]), xs[2]),
           "max": torch.maximum(torch.maximum(xs[0], xs[1]), xs[2]), "avg": (xs[0] + xs[1] + xs[2]) / 3}[op]
    torch.testing.assert_close(got, exp)


def test_reduce_reference_int_and_bool():
    a, b = torch.tensor([6, 3, -7]), torch.tensor([3, 5, 2])
    assert torch.equal(ops.reduce_nway_reference([a, b], "band"), a & b)
    assert torch.equal(ops.reduce_nway_reference([a, b], "bxor"), a ^ b)
    assert torch.equal(ops.reduce_nway_reference([a, b], "avg"), torch.tensor([4, 4, -2]))
    t, f = torch.tensor([True, False]), torch.tensor([True, True])
    assert torch.equal(ops.reduce_nway_reference([t, f], "sum"), t | f)


def test_native_extension_loads_and_registers():
    import torch.distributed as dist

    import pytorch_distributed_collective_communication_amd as pdcc

    C = pdcc._load_native()
    assert issubclass(C.ProcessGroupMI355X, torch._C._distributed_c10d.Backend)
    assert "MI355X" in dist.Backend._plugins
    assert C.TILE_BYTES == 4096 and C.MAX_RANKS_IPC == 8


def test_ops_reject_cpu_tensors():
    with pytest.raises(RuntimeError):
        ops.reduce_nway([torch.ones(4), torch.ones(4)])


def test_flight_recorder():
    recs, dump = launch(W.flight_probe, 2)[0]
    ops_ = [r["op"] for r in recs]
    assert ops_[-4:] == ["allreduce/shm"] * 3 + ["broadcast/shm"]
    assert all(r["state"] == "done" for r in recs)
    assert "flight recorder" in dump and "broadcast/shm" in dump


def test_rccl_env_forwarding():
    # PDCC_RCCL_* -> NCCL_* before the first communicator, once per process; the user's own
    # NCCL_* setting wins (verdict r1: tuning hooks for 7 xGMI links)
    import subprocess
    import sys

    code = ("import ctypes, pytorch_distributed_collective_communication_amd as p; C = p._load_native(); "
            "g = ctypes.CDLL(None).getenv; g.restype = ctypes.c_char_p; "
            "print(sorted(C.forwarded_rccl_env())); "
            "print(*[(g(k.encode()) or b'None').decode() for k in ('NCCL_BUFFSIZE', 'NCCL_PROTO', 'NCCL_MIN_NCHANNELS')])")
    env = {k: v for k, v in os.environ.items() if not k.startswith(("NCCL_", "PDCC_RCCL_"))}
    env.update({"PDCC_RCCL_BUFFSIZE": "8388608", "PDCC_RCCL_PROTO": "Simple", "PDCC_RCCL_MIN_NCHANNELS": "28",
                "NCCL_PROTO": "LL128"})
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert lines[-2] == "['NCCL_BUFFSIZE=8388608', 'NCCL_MIN_NCHANNELS=28']", lines
    assert lines[-1] == "8388608 LL128 28", lines


@pytest.mark.parametrize("env", [{}, {"PDCC_IPC_ZC": "0", "PDCC_IPC_ZC_MIN": "4M", "PDCC_IPC_PUSH": "0",
                                       "PDCC_IPC_ZC_CACHE": "3", "PDCC_ALGO": "ipc_push",
                                       "PDCC_RCCL_WIDE_CTAS": "56", "PDCC_RCCL_WIDE_MIN": "64M",
                                       "PDCC_IPC_GRID": "1024", "PDCC_IPC_WIDE_GRID": "0",
                                       "PDCC_IPC_LL_MAX": "4K", "PDCC_IPC_SDMA": "0", "PDCC_SDMA_STREAMS": "5",
                                       "PDCC_IPC_ZC_SIZE_GUARD": "0"}])
def test_python_config_mirror_matches_the_backend(env):
    # the Python mirror (config.py) and the C++ Config read the same variables with the same defaults
    import re

    from pytorch_distributed_collective_communication_amd.parallel.spawn import launch
    from tests import _workers as W

    desc, py = launch(W.config_probe, 1, env=env)[0]
    cpp = dict(re.findall(r"(\w+)=(\S+)", desc))
    for key in ("ipc_1shot_max", "ipc_2shot_max", "ipc_copy_max", "ipc_max_staging", "ipc_zc", "ipc_zc_min",
                "ipc_zc_cache", "ipc_push", "ipc_spin_ms", "ipc_grid", "ipc_wide_grid", "ipc_ll_max", "autotune", "autotune_sample", "algo",
                "rccl_wide_ctas", "rccl_wide_min", "a2a_list_agree", "ipc_zc_async", "ipc_sdma", "sdma_streams",
                "ipc_zc_size_guard"):
        want = py[key]
        got = cpp[key].rstrip(",)")
        assert got == (str(int(want)) if isinstance(want, bool) else str(want)), (key, got, want)


def test_issue_order_bookkeeping_dry():
    # RcclComm's cross-stream issue order (csrc/device/issue_order.h) without a GPU: the stream
    # operations it would issue, for one group (lazy ticks) and after a second group shares it
    import pytorch_distributed_collective_communication_amd as pdcc

    C = pdcc._load_native()
    o = C.IssueOrder(dry=True)
    for s in (1, 1):  # same stream: FIFO already, nothing to issue
        o.enter(s)
        o.leave(s)
    assert o.log() == [] and o.waits() == 0
    o.enter(2)  # switch: tick the previous stream lazily, wait for it
    o.leave(2)
    assert o.log() == ["write 1 1", "wait 2 1"] and o.waits() == 1
    o.add_user()  # shared: every op ticks right after itself
    o.enter(2)
    o.leave(2)
    o.enter(1)
    o.leave(1)
    assert o.log()[2:] == ["write 2 2", "wait 1 2", "write 1 3"], o.log()
    assert o.users() == 2 and o.ticks() == 3 and o.waits() == 2


def test_conformance_helpers():
    # the bench's conformance pass: engine patterns and the fp64-referenced closeness rule
    import torch

    from pytorch_distributed_collective_communication_amd.utils import conformance as cf

    assert cf._engine_matches("ipc_2shot_dyn_zc", "ipc_2shot_dyn*")
    assert cf._engine_matches("rccl_wide", "rccl*") and cf._engine_matches("anything", "*")
    assert not cf._engine_matches("ipc_2shot", "ipc_2shot_zc")
    xs = [torch.tensor([1.0, -2.0, 3.0]) * (r + 1) for r in range(4)]
    assert cf._close(sum(xs), xs, "SUM", 4, "float32")
    assert not cf._close(sum(xs) + 1e-3, xs, "SUM", 4, "float32")
    assert cf._close(torch.stack(xs).amax(0), xs, "MAX", 4, "float32")
    assert cf._close(sum(xs) / 4, xs, "AVG", 4, "float32")
    assert cf._close(torch.stack(xs).prod(0), xs, "PRODUCT", 4, "float32")
    b = [x.to(torch.bfloat16) for x in xs]
    assert cf._close(sum(x.float() for x in b).to(torch.bfloat16), b, "SUM", 4, "bfloat16")


def test_conformance_zero_copy_check_fails_on_a_fallback():
    # verdict r5 Next #1: a "*_zc" expectation fails when any call of the check ran staged, even if the
    # label of its last call says zero-copy; the delta is in the record
    from pytorch_distributed_collective_communication_amd.utils import conformance as cf

    class FakeBackend:
        def __init__(self, label, fallback_per_call):
            self.label, self.step, self.n = label, fallback_per_call, 0

        def last_algo(self):
            return self.label

        def zc_counters(self):
            return {"zc_calls": 5, "zc_fallbacks": self.n}

        def run(self):
            self.n += self.step
            return True

    P = cf._Pass(0, 1, "cpu", deadline_s=60)
    ok_b, bad_b, lab_b = FakeBackend("ipc_2shot_zc", 0), FakeBackend("ipc_2shot_zc", 1), FakeBackend("ipc_2shot", 0)
    P.check("zc/ok", ok_b, ok_b.run, expect_engine="ipc_2shot_zc")
    P.check("zc/fell_back", bad_b, bad_b.run, expect_engine="ipc_2shot_zc")
    P.check("zc/staged_label", lab_b, lab_b.run, expect_engine="ipc_2shot_zc")
    P.check("staged/any", bad_b, bad_b.run, expect_engine="ipc_2shot")  # (not a zero-copy expectation)
    r = P.result()
    assert r["checks"]["zc/ok"] == {"ok": True, "engine": "ipc_2shot_zc", "want": "ipc_2shot_zc", "zc_fallbacks": 0}
    assert r["checks"]["zc/fell_back"]["ok"] is False and r["checks"]["zc/fell_back"]["zc_fallbacks"] == 1
    assert r["checks"]["zc/staged_label"]["ok"] is False
    assert r["checks"]["staged/any"]["ok"] is False  # (label "ipc_2shot_zc" is not "ipc_2shot")
    assert sorted(r["failed"]) == ["staged/any", "zc/fell_back", "zc/staged_label"]
