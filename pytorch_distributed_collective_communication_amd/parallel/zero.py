"""ZeRO-style sharded data parallelism on the mi355x backend.

The reference motivates ``all_gather`` with "have a copy of the information on
all the devices" (README.md:254) and data parallelism with gradient averaging
(README.md:5); BASELINE.json names the ZeRO-style parameter gather (bf16
``all_gather`` of 4 GiB per rank on 8 GPUs) as one of its configs. This module
is that workload: :class:`ShardedOptimizer` keeps ONE full copy of the
parameters for forward/backward but only 1/world of the optimizer state and
fp32 master weights per rank, and each step is

1. ``reduce_scatter_tensor`` (``ReduceOp.AVG``: divided inside the reduction on
   mi355x) of each gradient bucket -> this rank's shard of the bucket, launched
   with ``async_op=True`` the moment backward has produced the bucket's last
   gradient (``register_post_accumulate_grad_hook``), so the reduction overlaps
   the rest of the backward pass;
2. the inner optimizer's step on this rank's (fp32) master shard only;
3. ``all_gather_into_tensor`` of the updated shards (in the parameter dtype,
   e.g. bf16) straight back into the flat parameter buffer, one per bucket.

MI355X-first layout: every parameter of one (device, dtype) is a view into one
flat buffer (and its ``.grad`` a view into one flat gradient buffer, which
autograd accumulates into in place), laid out in backward order and cut into
buckets of ``bucket_bytes`` (default 256 MiB: large messages keep RCCL and the
IPC kernels over xGMI on their bandwidth plateau). No pack/unpack copies: the
collectives read and write the buffers the model uses. Buckets are padded to a
multiple of ``world x 64`` elements so every shard is 16-byte aligned (zero-copy
IPC). With 288 GB of HBM per GPU the full parameter copy is cheap; what sharding
saves is the optimizer state (2 fp32 words per parameter for Adam) and the
master weights.

Gradient accumulation: backward passes inside ``with opt.no_sync():`` only
accumulate; a second backward outside it before :meth:`step` raises instead of
double-reducing a bucket.

``state_dict()`` / ``load_state_dict()`` save and restore this rank's shard
(sharded checkpoint: every rank writes its own file) and re-gather the
parameters on load.
"""
from __future__ import annotations

import contextlib
import copy
from typing import Dict, Iterable, List

import torch
import torch.distributed as dist

_ALIGN = 64  # elements; x world = padding unit of every bucket


class _Bucket:
    """A contiguous range [off, off + padded) of one flat space; this rank owns
    [off + rank * shard, off + (rank + 1) * shard) of it, stored at
    [soff, soff + shard) of the space's shard buffers."""

    def __init__(self, idx: List[int], off: int, padded: int, world: int, soff: int):
        self.idx, self.off, self.padded = idx, off, padded
        self.shard = padded // world
        self.soff = soff
        self.pending = len(idx)
        self.work = None


class _FlatSpace:
    """All parameters of one (device, dtype): flat params, flat grads, buckets, this rank's shards."""

    def __init__(self, params: List[torch.nn.Parameter], world: int, rank: int, master_dtype, bucket_bytes: int):
        p0 = params[0]
        self.params = params  # backward order
        self.dtype, self.device = p0.dtype, p0.device
        unit = world * _ALIGN
        esize = p0.element_size()
        self.offsets = []
        self.buckets: List[_Bucket] = []
        off = soff = 0
        cur, cur_n = [], 0

        def close():
            nonlocal off, soff, cur, cur_n
            padded = (cur_n + unit - 1) // unit * unit
            b = _Bucket(cur, off, padded, world, soff)
            self.buckets.append(b)
            off += padded
            soff += b.shard
            cur, cur_n = [], 0

        for i, p in enumerate(params):
            if cur and (cur_n + p.numel()) * esize > bucket_bytes:
                close()
            self.offsets.append(off + cur_n)
            cur.append(i)
            cur_n += p.numel()
        close()
        self.where = {}
        for bi, b in enumerate(self.buckets):
            for i in b.idx:
                self.where[id(params[i])] = bi
        self.padded, self.shard_total = off, soff
        self.rank = rank
        with torch.no_grad():
            self.flat = torch.zeros(off, dtype=self.dtype, device=self.device)
            self.grad = torch.zeros(off, dtype=self.dtype, device=self.device)
            for p, o in zip(params, self.offsets):
                self.flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
            self.attach()
            self.grad_shard = torch.empty(soff, dtype=self.dtype, device=self.device)
            self.param_shard = torch.empty(soff, dtype=self.dtype, device=self.device)
            for b in self.buckets:
                self.param_shard[b.soff:b.soff + b.shard].copy_(self.own(self.flat, b))
            md = master_dtype if self.dtype.is_floating_point else self.dtype
            self.master = self.param_shard.to(md).clone()

    def own(self, buf: torch.Tensor, b: _Bucket) -> torch.Tensor:
        lo = b.off + self.rank * b.shard
        return buf[lo:lo + b.shard]

    def attach(self) -> None:
        """(Re)point every parameter and its ``.grad`` at the flat buffers."""
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            p.data = self.flat[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)

    def sync_grads_in(self, b: _Bucket) -> None:
        """Gradients replaced behind our back (``set_to_none``, manual assignment) are
        copied into the flat buffer and re-attached."""
        for i in b.idx:
            p, o = self.params[i], self.offsets[i]
            view = self.grad[o:o + p.numel()]
            if p.grad is None:
                view.zero_()
            elif p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad.reshape(-1))
            p.grad = view.view_as(p)


class ShardedOptimizer:
    """ZeRO-style (optimizer state + master weights sharded) data-parallel optimizer.

    Usage::

        opt = ShardedOptimizer(model.parameters(), torch.optim.AdamW, lr=1e-3)
        for x, y in batches:             # this rank's batch shard
            loss_fn(model(x), y).backward()   # bucket reduce-scatters start here
            opt.step()                    # wait, sharded step, all-gather
            opt.zero_grad()

    ``broadcast_from`` (default 0) makes every replica start from that rank's
    parameters; ``master_dtype`` (default fp32) is the dtype of the sharded
    master weights and optimizer state for floating-point parameters -- with
    bf16 parameters the optimizer math runs in fp32 and only the gathered
    parameters are bf16. ``overlap=False`` defers every reduce-scatter to
    :meth:`step`. One parameter group: the inner optimizer's hyper-parameters
    come from ``**opt_kwargs``.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], optimizer_cls=torch.optim.SGD, group=None,
                 master_dtype: torch.dtype = torch.float32, broadcast_from: int | None = 0,
                 bucket_bytes: int = 256 << 20, overlap: bool = True, **opt_kwargs):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("ShardedOptimizer: no parameters that require grad")
        if broadcast_from is not None:
            src = dist.get_global_rank(group, broadcast_from) if group is not None else broadcast_from
            with torch.no_grad():
                for p in params:
                    dist.broadcast(p.data, src=src, group=group)
        by_key: Dict[tuple, List[torch.nn.Parameter]] = {}
        for p in reversed(params):  # ~ the order backward produces gradients
            by_key.setdefault((str(p.device), p.dtype), []).append(p)
        self.spaces = [_FlatSpace(ps, self.world, self.rank, master_dtype, bucket_bytes) for ps in by_key.values()]
        self._space_of = {id(p): s for s in self.spaces for p in s.params}
        self.inner = optimizer_cls([s.master for s in self.spaces], **opt_kwargs)
        self._avg = self._fused_avg()
        self._op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        self._sync = True
        self.overlapped = 0  # buckets whose reduce-scatter started during backward (last step())
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params] if overlap else []

    def _fused_avg(self) -> bool:
        """mi355x divides inside the reduction (ReduceOp.AVG); others get SUM + one scale."""
        try:
            from .backend import native_backend

            native_backend(self.group, self.spaces[0].device.type)
            return True
        except Exception:
            return False

    @property
    def param_groups(self):
        return self.inner.param_groups

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes in this context accumulate gradients locally (no communication)."""
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def _launch(self, s: _FlatSpace, b: _Bucket) -> None:
        s.sync_grads_in(b)
        b.work = dist.reduce_scatter_tensor(s.grad_shard[b.soff:b.soff + b.shard], s.grad[b.off:b.off + b.padded],
                                            op=self._op, group=self.group, async_op=True)

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        if not self._sync:
            return
        s = self._space_of[id(p)]
        b = s.buckets[s.where[id(p)]]
        if b.pending <= 0:
            raise RuntimeError(
                "ShardedOptimizer: a gradient arrived for a bucket that is already being reduced -- two backward "
                "passes without step() in between; wrap the accumulation steps in `with opt.no_sync():`")
        b.pending -= 1
        if b.pending == 0:
            with torch.no_grad():
                self._launch(s, b)

    def zero_grad(self, set_to_none: bool = False) -> None:  # noqa: ARG002 - the flat buffer stays attached
        for s in self.spaces:
            s.grad.zero_()
            s.attach()

    @torch.no_grad()
    def step(self) -> None:
        self.overlapped = sum(b.work is not None for s in self.spaces for b in s.buckets)
        for s in self.spaces:
            for b in s.buckets:
                if b.work is None:  # not launched during backward (overlap off, unused params)
                    self._launch(s, b)
        for s in self.spaces:
            for b in s.buckets:
                b.work.wait()
                b.work = None
                b.pending = len(b.idx)
            g = s.grad_shard if s.master.dtype == s.dtype else s.grad_shard.to(s.master.dtype)
            if not self._avg and self.world > 1:
                g = g / self.world
            s.master.grad = g
        self.inner.step()
        self._gather()

    @torch.no_grad()
    def _gather(self) -> None:
        works = []
        for s in self.spaces:
            s.param_shard.copy_(s.master)
            for b in s.buckets:
                works.append(dist.all_gather_into_tensor(s.flat[b.off:b.off + b.padded],
                                                         s.param_shard[b.soff:b.soff + b.shard],
                                                         group=self.group, async_op=True))
        for w in works:
            w.wait()

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []

    # ---- sharded checkpoint / resume
    def _layout(self):
        return [(str(s.dtype), [(b.off, b.padded) for b in s.buckets]) for s in self.spaces]

    def state_dict(self) -> dict:
        """This rank's shard: master weights + inner optimizer state (+ layout check)."""
        return {
            "world": self.world,
            "rank": self.rank,
            "layout": self._layout(),
            "master": [s.master.detach().clone() for s in self.spaces],
            "inner": copy.deepcopy(self.inner.state_dict()),  # a snapshot, not live state
        }

    @torch.no_grad()
    def load_state_dict(self, sd: dict) -> None:
        if sd["world"] != self.world or sd["rank"] != self.rank:
            raise ValueError(f"ShardedOptimizer: checkpoint is rank {sd['rank']}/{sd['world']}, "
                             f"this is rank {self.rank}/{self.world}")
        if sd["layout"] != self._layout():
            raise ValueError("ShardedOptimizer: checkpoint parameter layout differs from this model's")
        for s, m in zip(self.spaces, sd["master"]):
            s.master.copy_(m)
        self.inner.load_state_dict(sd["inner"])
        self._gather()

    def sharded_state_bytes(self) -> int:
        """Bytes of master weights + optimizer state held by this rank."""
        n = sum(s.master.numel() * s.master.element_size() for s in self.spaces)
        for st in self.inner.state.values():
            for v in st.values():
                if torch.is_tensor(v):
                    n += v.numel() * v.element_size()
        return n


__all__ = ["ShardedOptimizer"]
