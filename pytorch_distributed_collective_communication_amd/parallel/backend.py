"""Registration of the ``mi355x`` c10d backend with ``torch.distributed``.

The reference selects its backend with ``dist.init_process_group("gloo", ...)``
(reference main.py:90,94) and builds sub-groups with ``dist.new_group``
(main.py:11,21,31,46,63,75). This module plugs the native
``ProcessGroupMI355X`` (csrc/backend) into that unchanged front-end:

* :func:`register` calls ``Backend.register_backend("mi355x", ..., extended_api=True,
  devices=["cpu", "cuda"])`` so ``init_process_group("mi355x")`` and every
  ``new_group()`` of that world build our backend for CPU *and* GPU tensors;
* :func:`install_takeover` optionally rebinds ``torch.distributed.init_process_group``
  so a literal ``"gloo"`` (or ``"nccl"``) request is served by ``mi355x`` --
  this is how the reference's ``main.py`` runs unmodified on this library
  (``PDCC_TAKEOVER_GLOO=1``, set by ``python -m <pkg>.run``).
"""
from __future__ import annotations

import functools
import os
import threading

BACKEND_NAME = "mi355x"
_lock = threading.RLock()
_registered = False
_takeover: set[str] = set()
_orig_init = None


def _native():
    from .. import _load_native

    C = _load_native()
    if not hasattr(C.ProcessGroupMI355X, "options"):
        C.ProcessGroupMI355X.options = property(_backend_options)
    return C


_options_cls = None


def _backend_options(backend):
    """``backend.options`` (torch's split_group deep-copies the parent's): a c10d
    Backend.Options carrying this group's timeout, deep-copyable."""
    global _options_cls
    import datetime

    import torch

    if _options_cls is None:
        base = torch._C._distributed_c10d.Backend.Options

        class _Options(base):
            def __deepcopy__(self, memo):
                o = _Options(self.backend, self._timeout)
                o.group_name = self.group_name
                return o

        _options_cls = _Options
    return _options_cls(BACKEND_NAME, datetime.timedelta(milliseconds=backend.timeout_ms()))


_bound = False


def bind_local_rank() -> int | None:
    """``run.py --nproc`` ranks (PDCC_BIND_LOCAL_RANK=1): make GPU ``LOCAL_RANK % count`` this process's
    device at its first process group, unless the script already picked one. Returns the device bound."""
    global _bound
    if _bound or os.environ.get("PDCC_BIND_LOCAL_RANK") != "1":
        return None
    _bound = True
    import torch

    n = torch.cuda.device_count()  # (does not initialise the GPU on this runtime)
    if n == 0:
        return None
    if torch.cuda.is_initialized() and torch.cuda.current_device() != 0:
        return None  # the script chose its device itself
    d = int(os.environ.get("LOCAL_RANK", "0")) % n
    torch.cuda.set_device(d)
    return d


def _create(dist_opts, backend_opts):
    C = _native()
    bind_local_rank()
    # an earlier RCCL environment sweep's verdict for this topology (utils/rccl_env.py), before the
    # process's first RCCL communicator reads its environment
    from ..utils import rccl_env

    try:
        rccl_env.apply_persisted(int(dist_opts.group_size))
    except Exception:  # (a malformed file never stops a group from coming up)
        pass
    return C.ProcessGroupMI355X(
        dist_opts.store,
        dist_opts.group_rank,
        dist_opts.group_size,
        dist_opts.timeout,
        list(dist_opts.global_ranks_in_group or []),
        str(dist_opts.group_id or ""),
    )


def register() -> None:
    """Register the ``mi355x`` backend (idempotent, cheap: the native library is
    only loaded when the first process group is created)."""
    global _registered
    if _registered:
        return
    # Import OUTSIDE the lock: the first `import torch` runs torch's backend
    # autoload hook, which re-enters register() through _autoload.
    import torch.distributed as dist

    with _lock:
        if _registered:
            return
        if BACKEND_NAME.upper() not in getattr(dist.Backend, "_plugins", {}):
            dist.Backend.register_backend(BACKEND_NAME, _create, extended_api=True, devices=["cpu", "cuda"])
        _registered = True


def _map_backend(backend):
    if isinstance(backend, str) and backend.lower() in _takeover:
        return BACKEND_NAME
    return backend


def install_takeover(names=("gloo",)) -> None:
    """Serve ``init_process_group(<name>)`` requests for ``names`` with ``mi355x``."""
    global _orig_init
    import torch.distributed as dist
    import torch.distributed.distributed_c10d as c10d

    register()
    with _lock:
        _takeover.update(n.lower() for n in names)
        if _orig_init is not None:
            return
        _orig_init = c10d.init_process_group

        @functools.wraps(_orig_init)
        def init_process_group(backend=None, *args, **kwargs):
            return _orig_init(_map_backend(backend), *args, **kwargs)

        init_process_group.__pdcc_takeover__ = True
        dist.init_process_group = init_process_group
        c10d.init_process_group = init_process_group


def takeover_from_env() -> None:
    names = []
    if os.environ.get("PDCC_TAKEOVER_GLOO", "0") not in ("", "0"):
        names.append("gloo")
    if os.environ.get("PDCC_TAKEOVER_NCCL", "0") not in ("", "0"):
        names.append("nccl")
    if names:
        install_takeover(names)


def native_backend(group=None, device=None):
    """The ``ProcessGroupMI355X`` object behind ``group`` (default: world)."""
    import torch
    import torch.distributed as dist

    pg = group if group is not None else dist.group.WORLD
    dev = torch.device(device) if device is not None else torch.device("cpu")
    b = pg._get_backend(dev)
    C = _native()
    if not isinstance(b, C.ProcessGroupMI355X):
        raise RuntimeError(f"group is not served by the {BACKEND_NAME} backend (got {type(b).__name__})")
    return b


def stats(group=None) -> dict:
    """Per (collective/algorithm) counters: {key: (calls, bytes, host_ms)}."""
    return dict(native_backend(group).stats())


def last_algo(group=None) -> str:
    return native_backend(group).last_algo()


def zc_counters(group=None) -> dict:
    """Zero-copy outcomes of the group's GPU calls: ``zc_calls`` (ran zero-copy), ``zc_fallbacks``
    (attempted, ran staged), plus the export refusals (size guard, full mapping list)."""
    return dict(native_backend(group, "cuda").zc_counters())


def describe(group=None) -> str:
    return native_backend(group).describe()


def autotune_table(group=None) -> list:
    """Decisions of the online autotuner so far (one dict per collective and
    power-of-two size bucket: reference-engine and IPC times, whether the IPC
    result matched, and the adopted engine). See PDCC_AUTOTUNE in config.py."""
    return native_backend(group).autotune_table()
