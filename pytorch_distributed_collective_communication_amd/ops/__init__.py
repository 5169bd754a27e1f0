"""Tensor-level access to the gfx950 kernels.

* :func:`reduce_nway` -- K1: ``out = op(srcs[0], ..., srcs[k-1])`` for 1..8
  same-shaped GPU tensors; ``op`` in sum/avg/prod/min/max (+ band/bor/bxor for
  integers). Default implementation stages tiles through LDS with
  ``global_load_lds_dwordx4`` (LDS-DMA ring); ``impl="regs"`` is the
  register-staged variant kept for A/B measurement; a ``_nt`` suffix
  (``"lds_nt"``, ``"regs_nt"``) makes the destination stores non-temporal.
* :func:`multi_copy`, :func:`pack`, :func:`unpack` -- K2: one launch copies a
  whole list of tensors (the staging used by gather/scatter/all_gather with
  tensor lists, reference main.py:35-37,51-52,66-68).

Every function runs on the current HIP stream and raises if the native
extension is missing (no silent eager fallback). ``*_reference`` functions are
the plain-PyTorch fp32 references the tests compare against.
"""
from __future__ import annotations

from typing import Sequence

import torch

_OPS = ("sum", "avg", "prod", "min", "max", "band", "bor", "bxor")


def _C():
    from .. import _load_native

    return _load_native()


# K1 variants (csrc/kernels/kernel_api.h K1Mode): the LDS-DMA pipeline, the register pipeline,
# the streaming kernel (one slab per workgroup, grid over the whole buffer); `_nt` =
# non-temporal stores, `_ntl` = non-temporal loads and stores
K1_IMPLS = {"lds": 1, "regs": 0, "lds_nt": 3, "regs_nt": 2, "lds_ntl": 11, "regs_ntl": 10, "stream": 4,
            "stream_nt": 6, "stream_ntl": 14}


def reduce_nway(srcs: Sequence[torch.Tensor], out: torch.Tensor | None = None, op: str = "sum",
                impl: str = "lds_ntl", max_blocks: int = 0) -> torch.Tensor:
    """K1 N-way element-wise reduction on the GPU (1 <= len(srcs) <= 8).

    Default: the LDS-DMA pipeline with non-temporal loads and stores (6.27 TB/s for 2 fp32
    sources of 256 MiB on MI355X vs 6.06 for ``torch.add``, profiles/r3/k1_sweep_ntl_r3.json);
    ``stream_ntl`` is the fastest variant there (6.48 TB/s)."""
    if op not in _OPS:
        raise ValueError(f"op must be one of {_OPS}, got {op!r}")
    if impl not in K1_IMPLS:
        raise ValueError(f"impl must be one of {sorted(K1_IMPLS)}, got {impl!r}")
    srcs = list(srcs)
    if not srcs:
        raise ValueError("reduce_nway needs at least one source")
    if out is None:
        out = torch.empty_like(srcs[0], memory_format=torch.contiguous_format)
    _C().reduce_nway(srcs, out, op, K1_IMPLS[impl], int(max_blocks))
    return out


def reduce_nway_reference(srcs: Sequence[torch.Tensor], op: str = "sum") -> torch.Tensor:
    """Plain-PyTorch reference of :func:`reduce_nway` (f32 accumulation for floats)."""
    srcs = list(srcs)
    dt = srcs[0].dtype
    fl = dt.is_floating_point
    acc = srcs[0].to(torch.float64 if dt == torch.float64 else torch.float32) if fl else srcs[0].clone()
    for s in srcs[1:]:
        s2 = s.to(acc.dtype)
        if op in ("sum", "avg"):
            acc = acc + s2 if dt != torch.bool else (acc | s2)
        elif op == "prod":
            acc = acc * s2 if dt != torch.bool else (acc & s2)
        elif op == "max":
            acc = torch.maximum(acc, s2)
        elif op == "min":
            acc = torch.minimum(acc, s2)
        elif op == "band":
            acc = acc & s2
        elif op == "bor":
            acc = acc | s2
        elif op == "bxor":
            acc = acc ^ s2
    if op == "avg":
        acc = acc / len(srcs) if fl else torch.div(acc, len(srcs), rounding_mode="trunc")
    return acc.to(dt)


def multi_copy(srcs: Sequence[torch.Tensor], dsts: Sequence[torch.Tensor], max_blocks: int = 0,
               depth: int = 0, ntl: bool | None = None) -> None:
    """K2: copy srcs[i] -> dsts[i] for every i in ONE kernel launch.

    ``max_blocks`` caps the grid and ``depth`` (4 or 8) sets the LDS-DMA ring
    depth; 0 keeps the tuned defaults (csrc/kernels/kernel_api.h kK2Grid/kK2Depth); ``ntl``
    forces non-temporal source loads on / off (None: by the list's shape, see k2_ntl in copy.hip)."""
    _C().multi_copy(list(srcs), list(dsts), max_blocks, depth, -1 if ntl is None else int(bool(ntl)))


def _byte_view(t: torch.Tensor) -> torch.Tensor:
    return t.reshape(-1).view(torch.uint8)


def pack(tensors: Sequence[torch.Tensor], out: torch.Tensor | None = None) -> torch.Tensor:
    """Concatenate ``tensors`` (any dtypes) into one flat uint8 buffer with K2."""
    tensors = list(tensors)
    total = sum(t.numel() * t.element_size() for t in tensors)
    if out is None:
        out = torch.empty(total, dtype=torch.uint8, device=tensors[0].device)
    dsts, off = [], 0
    for t in tensors:
        n = t.numel() * t.element_size()
        dsts.append(out[off:off + n])
        off += n
    multi_copy([_byte_view(t) for t in tensors], dsts)
    return out


def unpack(flat: torch.Tensor, tensors: Sequence[torch.Tensor]) -> None:
    """Inverse of :func:`pack`: scatter a flat uint8 buffer back into ``tensors``."""
    tensors = list(tensors)
    srcs, off = [], 0
    for t in tensors:
        n = t.numel() * t.element_size()
        srcs.append(flat[off:off + n])
        off += n
    multi_copy(srcs, [_byte_view(t) for t in tensors])


__all__ = ["reduce_nway", "reduce_nway_reference", "multi_copy", "pack", "unpack"]
