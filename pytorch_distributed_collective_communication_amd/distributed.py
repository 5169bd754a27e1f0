"""Drop-in ``torch.distributed`` replacement (``import ... .distributed as dist``).

Same names and signatures as the calls the reference makes (main.py:5,11-94):
``init_process_group``, ``new_group``, ``ReduceOp``, ``reduce``, ``all_reduce``,
``scatter``, ``gather``, ``all_gather``, ``broadcast``, plus ``barrier``,
``get_rank``, ``get_world_size``, ``destroy_process_group`` and the rest of the
torch.distributed collective surface. The only behavioural difference: process
groups are served by the MI355X-native ``mi355x`` backend -- a literal
``"gloo"``/``"nccl"``/``None`` backend request is mapped to it.
"""
from __future__ import annotations

import torch.distributed as _td
from torch.distributed import *  # noqa: F401,F403 - re-export the full front-end

from .parallel.backend import BACKEND_NAME, describe, last_algo, register, stats  # noqa: F401

register()

ReduceOp = _td.ReduceOp
Backend = _td.Backend
group = _td.group

_MAPPED = {None, "gloo", "nccl", "cpu:gloo,cuda:nccl", BACKEND_NAME}


def _map(backend):
    if backend is None:
        return BACKEND_NAME
    if isinstance(backend, str) and backend.lower() in _MAPPED:
        return BACKEND_NAME
    return backend


def init_process_group(backend=None, init_method=None, timeout=None, world_size=-1, rank=-1, store=None,
                       group_name="", pg_options=None, device_id=None):
    """torch.distributed.init_process_group with ``backend`` served by mi355x."""
    kw = dict(init_method=init_method, world_size=world_size, rank=rank, store=store, group_name=group_name,
              pg_options=pg_options, device_id=device_id)
    if timeout is not None:
        kw["timeout"] = timeout
    return _td.init_process_group(_map(backend), **kw)


def new_group(ranks=None, timeout=None, backend=None, pg_options=None, use_local_synchronization=False,
              group_desc=None, device_id=None):
    """torch.distributed.new_group; sub-groups are mi355x groups too."""
    return _td.new_group(ranks=ranks, timeout=timeout, backend=_map(backend) if backend else None,
                         pg_options=pg_options, use_local_synchronization=use_local_synchronization,
                         group_desc=group_desc, device_id=device_id)


def is_mi355x_available() -> bool:
    from . import native_available

    return native_available()


def _pg(group):
    return group if group is not None else _td.distributed_c10d._get_default_group()


def all_gather_into_tensor_coalesced(outputs, inputs, group=None, async_op=False):
    """Every ``inputs[i]`` gathered into ``outputs[i]`` (``world x`` its size) as ONE collective:
    the backend packs the members, runs one all-gather and unpacks (csrc/backend/coalesced.cpp).
    The same call torch's ``_coalescing_manager`` makes, without recording each member in Python."""
    work = _pg(group).allgather_into_tensor_coalesced(list(outputs), list(inputs))
    if async_op:
        return work
    work.wait()


def reduce_scatter_tensor_coalesced(outputs, inputs, op=ReduceOp.SUM, group=None, async_op=False):
    """Chunk ``rank`` of every ``inputs[i]``, reduced over the group, into ``outputs[i]`` -- ONE collective."""
    opts = _td.ReduceScatterOptions()
    opts.reduceOp = op
    work = _pg(group).reduce_scatter_tensor_coalesced(list(outputs), list(inputs), opts)
    if async_op:
        return work
    work.wait()
