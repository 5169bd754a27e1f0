"""Python mirror of the backend's PDCC_* configuration (csrc/backend/config.h).

The native backend reads these environment variables once, when a process
group is constructed; :func:`current` shows what a new group would use and
:func:`env_for` builds an environment dict (e.g. for ``parallel.spawn.launch``).

| variable | default | meaning |
|---|---|---|
| PDCC_ALGO | auto | force ``rccl`` / ``rccl_wide`` / ``ipc`` / ``ipc_push`` / ``ipc_wide`` / ``ipc_staged`` (IPC without zero copy) / ``ipc_dyn`` (dynamic zero-copy 2-shot all-reduce) / ``ipc_sdma`` (copy collectives as copy-engine pulls between mapped user buffers) / ``host`` for GPU tensors (preferred if feasible) |
| PDCC_IPC | 1 | enable the hipIpc peer-memory path |
| PDCC_IPC_SELFTEST | 1 | run the IPC protocol once on known data when a group first uses a GPU; any failure on any rank disables IPC for that group |
| PDCC_IPC_SELFTEST_MS | 20000 | spin timeout of the self-test's cross-GPU barriers (capped by the group timeout) |
| PDCC_IPC_SELFTEST_FAIL | "" | test hook: this rank reports a failed self-test |
| PDCC_IPC_1SHOT_MAX | 512K | all-reduce/reduce/broadcast up to this size: 1-shot protocol |
| PDCC_IPC_2SHOT_MAX | 8M | ... up to this size: 2-shot; above: RCCL |
| PDCC_IPC_COPY_MAX | 1M | gather/scatter/all-gather/reduce-scatter/all-to-all up to this: IPC |
| PDCC_IPC_MAX_STAGING | 1G | staging bytes; larger calls are chunked |
| PDCC_IPC_SPIN_MS | 600000 | bound on one cross-GPU barrier spin of the IPC kernels (the group timeout applies if shorter) |
| PDCC_IPC_ZC_ASYNC | 1 | zero-copy calls exchange their buffer records on a per-device launcher thread: the caller's host never waits for its peers (0: inline exchange) |
| PDCC_IPC_LL_MAX | 256K | collectives up to this size per rank / chunk (max 256K) use the LL protocol (flag-tagged pushes into the peers' signal areas, no staging copy, no barrier); 0: off |
| PDCC_IPC_GRID | 512 | workgroup cap of the IPC kernels on distinct GPUs (1..1024; ranks sharing a GPU: 256 / W) |
| PDCC_IPC_ASYNC_GRID | 0 | opt-in workgroup cap of the IPC/LL launches of async collectives (comm stream, overlapped with compute): leaves CU slots to the overlapped kernels; with a cap set every rank must pass the same async_op to each collective (torch treats async_op as rank-local; PDCC_DEBUG=1 checks it) (0: no cap) |
| PDCC_IPC_ZC_SIZE_GUARD | 1 | zero-copy refuses buffers whose allocation size has bit 31 set (2-4 GiB, 6-8 GiB: a peer's mapping of them stalls on this ROCm image); they run staged, and PDCC_IPC_MAX_STAGING stays below 2 GiB |
| PDCC_IPC_ZX | 1 | gated zero-copy calls resolve the peers' buffers on the device (mapping table); every rank's setting is voted on (AND) at the group's first GPU use |
| PDCC_IPC_DYN | 3 | chunks per workgroup of the dynamic zero-copy 2-shot all-reduce (``ipc_dyn``: workgroups claim chunks from a counter, per-chunk ready words instead of a block-pairwise barrier), which the autotuner races for zero-copy all_reduce keys; 0: not raced; agreed group-wide (minimum) |
| PDCC_IPC_SDMA | 1 | the autotuner races the copy-engine engine (``ipc_sdma``: hipMemcpyAsync pulls between IPC-mapped user buffers, no CU kernel) for broadcast / all_gather / gather / scatter / all_to_all keys of zero-copy sizes |
| PDCC_SDMA_STREAMS | 2 | side streams one ``ipc_sdma`` call's pulls fan out over (0..6) |
| PDCC_IPC_DYN_MIN_ROWS | 0 (= 16) | rows (W tiles each) per item of the dynamic protocols, at least: every item is its own short pipeline, so small items make them latency-bound; agreed group-wide (minimum) |
| PDCC_IPC_WIDE_GRID | 1024 | workgroup cap of the ``ipc_wide`` all-reduce the autotuner races for bulk keys on distinct GPUs (0: off) |
| PDCC_AUTOTUNE | 1 | every GPU collective with two feasible engines: time both on the first call per (collective, dtype, op/layout, power-of-two size) key (IPC result checked against the reference engine's), adopt the faster on all ranks |
| PDCC_AUTOTUNE_MIN / _MAX | 64K / 4T | size range the autotuner covers (outside: the static thresholds) |
| PDCC_AUTOTUNE_SAMPLE | 1G | bytes per engine the tuning runs move (a prefix of the caller's data) |
| PDCC_AUTOTUNE_COLLS | all | comma list of collectives to tune (allreduce, reduce, broadcast, allgather, gather, scatter, reduce_scatter, alltoall) |
| PDCC_AUTOTUNE_SPIN_MS | 10000 | spin bound of IPC runs during tuning; a timeout drops IPC for that key and keeps the group healthy |
| PDCC_AUTOTUNE_FILE | "" | persisted decisions: keys with a line in this file (same topology signature on every rank) take the recorded engine without a race; rank 0 appends every new race's verdict |
| PDCC_RCCL_INIT_TIMEOUT_S | 300 | deadline of one RCCL communicator creation (non-blocking init / split, polled; capped by the group timeout): a peer that never joins fails the group with a clear error, later calls fail at once |
| PDCC_RCCL_NONBLOCKING | 1 | create RCCL communicators non-blocking (polled against the deadline above); 0: RCCL's blocking creation |
| PDCC_RCCL_MIN_CTAS / _MAX_CTAS | -1 / -1 | RCCL channel (CTA) bounds via ``ncclCommInitRankConfig``; -1 leaves RCCL's topology tuner in charge |
| PDCC_RCCL_GROUP_COMM | share | groups with the same members as a live communicator: share it, split from it (ncclCommSplit) or init a fresh one |
| PDCC_RCCL_SPLIT_SHARE | 1 | ncclCommSplit children share the parent's resources |
| PDCC_RCCL_BUFFSIZE / _ALGO / _PROTO / _MIN_NCHANNELS / _MAX_NCHANNELS / _NTHREADS / _MSCCL / _MSCCLPP | unset | forwarded to NCCL_* / RCCL_* before the process's first communicator (the user's own NCCL_* setting wins) |
| PDCC_LIST_GATHER | p2p | all_gather into separate tensors on RCCL: grouped send/recv into the list (p2p) or ring all_gather + K2 unpack (staged) |
| PDCC_A2A_LIST_AGREE | 1 | GPU ``all_to_all`` with tensor lists: the ranks agree (one host round) whether every chunk is equal, which unlocks the IPC/LL engines; 0: lists always use grouped point-to-point |
| PDCC_EAGER_INIT | 0 | build topology, IPC self-test and RCCL communicator when the group is created |
| PDCC_WORLD1_LOCAL | 1 | 1-rank groups short-circuit (0: still call RCCL, for tests) |
| PDCC_SHM_SLOT_BYTES | 8M | host transport staging slot per rank |
| PDCC_SHM_CHAN_BYTES | 1M | host transport p2p ring per directed pair |
| PDCC_SHM_SPIN_US | 300 | host transport busy-wait window before a futex sleep (20 when ranks > CPUs) |
| PDCC_XCHG_SPIN_US | 0 | the zero-copy exchange thread busy-waits this long for the next job before it sleeps (steady-state zero-copy calls resolve their buffers on the device, so the thread is off the critical path) |
| PDCC_STREAM | auto | GPU stream policy: auto (sync ops on the caller's stream, async on a comm stream), high, comm, current |
| PDCC_DEBUG | 0 | cross-rank fingerprint check before every collective |
| PDCC_LOG_LEVEL | 0 | 1: group/device info, 2: every collective |
| PDCC_BLOCKING_WAIT | 0 | ``Work.wait()`` blocks the host until the GPU op finished |
| PDCC_ROCTX | 0 | roctx range per collective (rocprofv3 --marker-trace) |
| PDCC_WATCHDOG_MS | 100 | watchdog poll period (0 disables timeout/abort handling) |
| PDCC_FLIGHT_RECORDER | 256 | number of recent collectives kept for post-mortem dumps |
| PDCC_FAULT | "" | fault injection ``rank:op_seq:kind`` (kind exit, raise, hang) |
| PDCC_TEST_AUTOTUNE_DELAY | "" | test hook ``rank:ms``: that rank starts its IPC tuning run late |
| PDCC_TEST_RCCL_INIT_SKIP / _RCCL_SHARED / _ZX_EPOCH | "" | test hooks: that rank never builds its communicator / claim RCCL on a shared GPU / start the device exchange epoch at this value |
| PDCC_TAKEOVER_GLOO / _NCCL | 0 | serve ``init_process_group("gloo"/"nccl")`` with mi355x |
"""
from __future__ import annotations

import os
from dataclasses import dataclass, fields

_SUFFIX = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}


def parse_bytes(v: str | int) -> int:
    if isinstance(v, int):
        return v
    v = v.strip()
    for suf in ("KiB", "MiB", "GiB"):
        if v.endswith(suf):
            v = v[:-3] + suf[0]
    if v and v[-1].upper() in _SUFFIX:
        return int(float(v[:-1]) * _SUFFIX[v[-1].upper()])
    return int(float(v))


@dataclass
class Config:
    algo: str = "auto"
    ipc: bool = True
    ipc_selftest: bool = True
    ipc_selftest_ms: int = 20000
    ipc_1shot_max: int = 512 << 10
    ipc_2shot_max: int = 8 << 20
    ipc_copy_max: int = 1 << 20
    ipc_max_staging: int = 1 << 30
    ipc_zc: bool = True
    ipc_push: bool = True
    ipc_dyn: int = 3
    ipc_dyn_min_rows: int = 0
    ipc_sdma: bool = True
    sdma_streams: int = 2
    ipc_zc_min: int = 1 << 20
    ipc_ll_max: int = 256 << 10
    ipc_zc_cache: int = 16
    ipc_zc_async: bool = True
    ipc_zx: bool = True
    ipc_zc_size_guard: bool = True
    ipc_async_grid: int = 0
    ipc_spin_ms: int = 600000
    ipc_grid: int = 512
    ipc_wide_grid: int = 1024
    autotune: bool = True
    autotune_min: int = 64 << 10
    autotune_max: int = 1 << 42
    autotune_sample: int = 1 << 30
    autotune_colls: str = "all"
    autotune_spin_ms: int = 10000
    autotune_file: str = ""
    rccl_init_timeout_s: int = 300
    rccl_nonblocking: bool = True
    rccl_min_ctas: int = -1
    rccl_max_ctas: int = -1
    rccl_wide_ctas: int = 112
    rccl_wide_min: int = 16 << 20
    rccl_group_comm: str = "share"
    rccl_split_share: bool = True
    list_gather: str = "p2p"
    a2a_list_agree: bool = True
    eager_init: bool = False
    world1_local: bool = True
    shm_slot_bytes: int = 8 << 20
    shm_chan_bytes: int = 1 << 20
    shm_spin_us: int = 300
    xchg_spin_us: int = 0
    stream: str = "auto"
    debug: bool = False
    log_level: int = 0
    blocking_wait: bool = False
    roctx: bool = False
    watchdog_ms: int = 100
    flight_recorder: int = 256
    fault: str = ""


_ENV = {
    "algo": "PDCC_ALGO", "ipc": "PDCC_IPC", "ipc_selftest": "PDCC_IPC_SELFTEST",
    "ipc_selftest_ms": "PDCC_IPC_SELFTEST_MS", "ipc_1shot_max": "PDCC_IPC_1SHOT_MAX",
    "ipc_2shot_max": "PDCC_IPC_2SHOT_MAX", "ipc_copy_max": "PDCC_IPC_COPY_MAX",
    "ipc_max_staging": "PDCC_IPC_MAX_STAGING", "ipc_zc": "PDCC_IPC_ZC", "ipc_push": "PDCC_IPC_PUSH", "ipc_dyn": "PDCC_IPC_DYN", "ipc_dyn_min_rows": "PDCC_IPC_DYN_MIN_ROWS", "ipc_sdma": "PDCC_IPC_SDMA", "sdma_streams": "PDCC_SDMA_STREAMS", "ipc_zc_min": "PDCC_IPC_ZC_MIN", "ipc_ll_max": "PDCC_IPC_LL_MAX",
    "ipc_zc_cache": "PDCC_IPC_ZC_CACHE", "ipc_zc_async": "PDCC_IPC_ZC_ASYNC",
    "ipc_zx": "PDCC_IPC_ZX", "ipc_zc_size_guard": "PDCC_IPC_ZC_SIZE_GUARD", "ipc_async_grid": "PDCC_IPC_ASYNC_GRID", "rccl_init_timeout_s": "PDCC_RCCL_INIT_TIMEOUT_S",
    "rccl_nonblocking": "PDCC_RCCL_NONBLOCKING", "autotune": "PDCC_AUTOTUNE",
    "autotune_min": "PDCC_AUTOTUNE_MIN", "autotune_max": "PDCC_AUTOTUNE_MAX", "world1_local": "PDCC_WORLD1_LOCAL",
    "ipc_spin_ms": "PDCC_IPC_SPIN_MS", "ipc_grid": "PDCC_IPC_GRID", "ipc_wide_grid": "PDCC_IPC_WIDE_GRID", "autotune_sample": "PDCC_AUTOTUNE_SAMPLE",
    "autotune_colls": "PDCC_AUTOTUNE_COLLS", "autotune_spin_ms": "PDCC_AUTOTUNE_SPIN_MS",
    "autotune_file": "PDCC_AUTOTUNE_FILE",
    "rccl_group_comm": "PDCC_RCCL_GROUP_COMM", "rccl_split_share": "PDCC_RCCL_SPLIT_SHARE",
    "list_gather": "PDCC_LIST_GATHER", "a2a_list_agree": "PDCC_A2A_LIST_AGREE", "eager_init": "PDCC_EAGER_INIT",
    "rccl_min_ctas": "PDCC_RCCL_MIN_CTAS", "rccl_max_ctas": "PDCC_RCCL_MAX_CTAS",
    "rccl_wide_ctas": "PDCC_RCCL_WIDE_CTAS", "rccl_wide_min": "PDCC_RCCL_WIDE_MIN",
    "shm_slot_bytes": "PDCC_SHM_SLOT_BYTES", "shm_chan_bytes": "PDCC_SHM_CHAN_BYTES",
    "shm_spin_us": "PDCC_SHM_SPIN_US", "xchg_spin_us": "PDCC_XCHG_SPIN_US", "stream": "PDCC_STREAM", "debug": "PDCC_DEBUG",
    "log_level": "PDCC_LOG_LEVEL", "blocking_wait": "PDCC_BLOCKING_WAIT", "roctx": "PDCC_ROCTX",
    "watchdog_ms": "PDCC_WATCHDOG_MS", "flight_recorder": "PDCC_FLIGHT_RECORDER", "fault": "PDCC_FAULT",
}


def _parse(field_type, raw: str):
    if field_type in (bool, "bool"):
        return raw.strip().lower() not in ("0", "false", "no", "off", "")
    if field_type in (int, "int"):
        return parse_bytes(raw)
    return raw


def current(environ=None) -> Config:
    """The configuration a process group created now would get."""
    env = os.environ if environ is None else environ
    c = Config()
    for f in fields(Config):
        raw = env.get(_ENV[f.name])
        if raw not in (None, ""):
            setattr(c, f.name, _parse(f.type, raw))
    if c.algo not in ("auto", "rccl", "rccl_wide", "ipc", "ipc_push", "ipc_wide", "ipc_staged", "ipc_dyn", "ipc_sdma",
                      "host"):
        raise ValueError("PDCC_ALGO must be auto|rccl|rccl_wide|ipc|ipc_push|ipc_wide|ipc_staged|ipc_dyn|ipc_sdma|host, "
                         f"got {c.algo!r}")
    if c.stream not in ("auto", "high", "comm", "current"):
        raise ValueError(f"PDCC_STREAM must be auto|high|comm|current, got {c.stream!r}")
    if c.rccl_group_comm not in ("share", "split", "init"):
        raise ValueError(f"PDCC_RCCL_GROUP_COMM must be share|split|init, got {c.rccl_group_comm!r}")
    if c.list_gather not in ("p2p", "staged"):
        raise ValueError(f"PDCC_LIST_GATHER must be p2p|staged, got {c.list_gather!r}")
    return c


def env_for(**overrides) -> dict:
    """Environment entries for the given overrides, e.g. ``env_for(algo="ipc", debug=True)``."""
    out = {}
    names = {f.name for f in fields(Config)}
    for k, v in overrides.items():
        if k not in names:
            raise KeyError(f"unknown PDCC config field {k!r}")
        out[_ENV[k]] = ("1" if v else "0") if isinstance(v, bool) else str(v)
    return out
