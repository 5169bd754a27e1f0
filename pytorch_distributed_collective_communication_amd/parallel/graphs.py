"""hipGraph capture of collectives on the mi355x backend.

A launch-bound sequence of collectives (the many small all-reduces of a decode
step, or of a data-parallel step with small buckets) costs more host time than
GPU time. On MI355X the remedy is a HIP graph, not a tracing compiler: capture
the sequence once with ``torch.cuda.graph`` and replay it with one launch.

What the backend does while the caller's stream is being captured
(csrc/backend/gpu_ops.cpp, csrc/device/ipc_comm.cpp, csrc/kernels/dev_common.h):

* every collective is enqueued on the capturing stream and returns an
  already-completed Work -- the graph node is the completion;
* the IPC kernels keep their call numbers on the device (per-block counters,
  csrc/kernels/kernel_api.h), never in a kernel argument (a graph replays
  arguments verbatim), so flag epochs advance on every replay exactly as for
  eager calls, and eager calls can be interleaved with replays;
* RCCL calls are captured as RCCL graph nodes;
* staging buffers a captured graph references are never freed while the group
  lives (a later, larger call grows into new buffers instead);
* what cannot be captured fails loudly: the host-staged engine, creating a
  communicator, growing the IPC staging, the autotuner's timing runs (an
  untuned size bucket uses the static choice while capturing).

:func:`capture` therefore runs ``fn`` eagerly ``warmup`` times first, which does
all of those once. The reference has no graphs (a CPU/Gloo tutorial,
main.py:1-108); this is the MI355X-native answer to launch-bound collective loops.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


class CollectiveGraph:
    """A captured sequence of collectives (plus any GPU work around them)."""

    def __init__(self, graph: torch.cuda.CUDAGraph, fn: Callable, result):
        self.graph = graph
        self.fn = fn
        self.result = result  # what fn returned during capture (its static output tensors, if any)

    def replay(self) -> None:
        """Enqueue one replay on the current stream (asynchronous, like the eager calls)."""
        self.graph.replay()

    __call__ = replay


def capture(fn: Callable[[], object], warmup: int = 2, group=None, stream: Optional[torch.cuda.Stream] = None,
            pool=None) -> CollectiveGraph:
    """Capture ``fn`` -- which issues collectives on static tensors -- into a graph.

    ``fn`` runs ``warmup`` times eagerly first (communicators, IPC staging, the
    autotuner's decisions), then once under capture. Every rank of the group
    must capture the same sequence of collectives and replay the graph the same
    number of times, in the same order relative to its eager collectives: the
    contract of the eager API.
    """
    s = stream if stream is not None else torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(max(0, warmup)):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier(group=group)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=pool, stream=s):
        out = fn()
    return CollectiveGraph(g, fn, out)
