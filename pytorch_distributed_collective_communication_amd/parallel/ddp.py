"""Data-parallel gradient synchronisation on the mi355x backend.

The reference motivates collectives with data parallelism: every worker
computes gradients on its batch shard and they are all-reduced and averaged
before the optimizer step (README.md:5), parameters/optimizer state are
broadcast to keep replicas identical (README.md:286) and batches are split
with scatter (README.md:182). :class:`GradBucketer` implements exactly that
contract, MI355X-first:

* gradients are packed into a few large flat buckets (default 256 MiB: big
  messages keep RCCL/IPC on their bandwidth plateau and 288 GB of HBM makes the
  extra copy cheap), filled in reverse registration order = backward order;
* each bucket is all-reduced with ``async_op=True`` the moment its last
  gradient is produced (``register_post_accumulate_grad_hook``), so
  communication overlaps the rest of the backward pass on the backend's
  high-priority comm stream;
* the average is fused into the reduction itself (``ReduceOp.AVG``: the IPC
  kernels divide in registers, RCCL uses ``ncclAvg``) on the mi355x backend --
  no separate pass over the buckets; other backends get SUM plus one scale;
* :meth:`finish` waits and unpacks every GPU bucket with ONE K2 ``multi_copy``
  launch (per-parameter copies on CPU);
* gradient accumulation: backward passes inside ``with bucketer.no_sync():``
  only accumulate into ``.grad``; the first backward after it launches the
  reduction of the accumulated gradients. A second backward before
  :meth:`finish` (outside ``no_sync``) raises instead of silently dropping a
  micro-batch.

``broadcast_parameters`` and ``scatter_batch`` cover the other two uses.
torch's own ``DistributedDataParallel`` also runs unchanged on this backend.
"""
from __future__ import annotations

import contextlib
from typing import Iterable, List

import torch
import torch.distributed as dist


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every replica identical to rank ``src`` (README.md:286)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)


def scatter_batch(batch: torch.Tensor | None, shard_shape, dtype, device, src: int = 0, group=None) -> torch.Tensor:
    """Split ``batch`` (on ``src``) along dim 0 into equal shards, one per rank (README.md:182)."""
    world = dist.get_world_size(group)
    out = torch.empty(shard_shape, dtype=dtype, device=device)
    chunks = list(batch.chunk(world, 0)) if dist.get_rank(group) == src else None
    if chunks is not None:
        chunks = [c.contiguous() for c in chunks]
    dist.scatter(out, scatter_list=chunks, src=src, group=group)
    return out


class _Bucket:
    def __init__(self, params: List[torch.nn.Parameter], dtype, device):
        self.params = params
        self.numel = sum(p.numel() for p in params)
        self.flat = torch.empty(self.numel, dtype=dtype, device=device)
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += p.numel()
        self.pending = 0
        self.work = None


class GradBucketer:
    """Overlapped, bucketed gradient all-reduce (average) for one module."""

    def __init__(self, module: torch.nn.Module, group=None, bucket_bytes: int = 256 << 20,
                 average: bool = True):
        self.group = group
        self.average = average
        self.world = dist.get_world_size(group)
        params = [p for p in module.parameters() if p.requires_grad]
        self.buckets: List[_Bucket] = []
        self._where = {}
        cur, cur_bytes = [], 0
        # reverse order ~ the order backward produces gradients
        for p in reversed(params):
            nb = p.numel() * p.element_size()
            if cur and (cur_bytes + nb > bucket_bytes or p.dtype != cur[0].dtype or p.device != cur[0].device):
                self._add_bucket(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            self._add_bucket(cur)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]
        self._sync = True
        self._fused_avg = average and self.world > 1 and _is_native(group, self.buckets)
        self._op = dist.ReduceOp.AVG if self._fused_avg else dist.ReduceOp.SUM
        self._reset()

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes in this context accumulate gradients locally (no communication)."""
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def _add_bucket(self, ps):
        b = _Bucket(ps, ps[0].dtype, ps[0].device)
        idx = len(self.buckets)
        for i, p in enumerate(ps):
            self._where[id(p)] = (idx, i)
        self.buckets.append(b)

    def _reset(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None

    def _on_grad(self, p: torch.nn.Parameter):
        if not self._sync:
            return
        bi, i = self._where[id(p)]
        b = self.buckets[bi]
        if b.pending <= 0:
            raise RuntimeError(
                "GradBucketer: a gradient arrived for a bucket that is already being reduced -- two backward "
                "passes without finish() in between; wrap the accumulation steps in `with bucketer.no_sync():`")
        off = b.offsets[i]
        b.flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
        b.pending -= 1
        if b.pending == 0:
            b.work = dist.all_reduce(b.flat, op=self._op, group=self.group, async_op=True)

    def finish(self) -> None:
        """Wait for every bucket, average, and write the result back into ``.grad``."""
        for b in self.buckets:
            if b.work is None:  # parameters without gradients this step: reduce what we have
                for p in b.params:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                for p, off in zip(b.params, b.offsets):
                    b.flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
                b.work = dist.all_reduce(b.flat, op=self._op, group=self.group, async_op=True)
        for b in self.buckets:
            b.work.wait()
            if self.average and self.world > 1 and not self._fused_avg:
                b.flat.div_(self.world)
            _unpack(b)
        self._reset()

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()


def _is_native(group, buckets) -> bool:
    """Is ``group`` served by the mi355x backend for the buckets' device (fused AVG)?"""
    if not buckets:
        return False
    try:
        from .backend import native_backend

        native_backend(group, buckets[0].flat.device.type)
        return True
    except Exception:
        return False


def _unpack(b: _Bucket) -> None:
    views = [b.flat[off:off + p.numel()] for p, off in zip(b.params, b.offsets)]
    grads = [p.grad.reshape(-1) if p.grad.is_contiguous() else None for p in b.params]
    if b.flat.is_cuda and all(g is not None for g in grads):
        try:
            from ..ops import multi_copy

            multi_copy(views, grads)  # one launch for the whole bucket
            return
        except Exception:  # extension unavailable: plain copies below
            pass
    for p, v in zip(b.params, views):
        p.grad.copy_(v.view_as(p.grad))


def allreduce_gradients(params: Iterable[torch.nn.Parameter], group=None, average: bool = True) -> None:
    """Non-overlapped reference implementation: one coalesced all-reduce per call."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    if average:
        flat.div_(dist.get_world_size(group))
    off = 0
    for g in grads:
        g.copy_(flat[off:off + g.numel()].view_as(g))
        off += g.numel()
