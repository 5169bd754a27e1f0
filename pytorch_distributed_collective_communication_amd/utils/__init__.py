"""Measurement helpers shared by bench.py, benchmarks/ and tests.

* :func:`busbw` / :func:`busbw_factor` -- nccl-tests bus-bandwidth convention
  (all_reduce 2(n-1)/n; reduce, broadcast 1; gather, scatter, all_gather,
  reduce_scatter, all_to_all (n-1)/n), used for every number in BASELINE.md;
* :func:`xgmi_ceiling_GBps` -- the link model of SURVEY.md §5.8 (an n-GPU group
  can use n-1 of the 7 xGMI links per GPU);
* :func:`p50` -- median of max-over-ranks latencies.
"""
from __future__ import annotations

import statistics
from typing import Iterable

XGMI_LINKS_PER_GPU = 7
XGMI_LINK_GBPS = 153.0  # per link, as used in SURVEY.md §5.8 / BASELINE.md §3

_FACTORS = {"all_reduce": lambda n: 2 * (n - 1) / n, "reduce": lambda n: 1.0, "broadcast": lambda n: 1.0}


def busbw_factor(coll: str, n: int) -> float:
    if n <= 1:
        return 0.0
    return _FACTORS.get(coll, lambda n: (n - 1) / n)(n)


def busbw(coll: str, nbytes: int, n: int, seconds: float) -> float:
    """Bus bandwidth in GB/s (1e9) for one collective of ``nbytes`` on ``n`` ranks."""
    if seconds <= 0:
        return 0.0
    return nbytes * busbw_factor(coll, n) / seconds / 1e9


def algbw(nbytes: int, seconds: float) -> float:
    return nbytes / seconds / 1e9 if seconds > 0 else 0.0


def xgmi_ceiling_GBps(n: int) -> float:
    """all_reduce busbw ceiling of an n-GPU group on one node (n-1 usable links)."""
    return max(0, min(n - 1, XGMI_LINKS_PER_GPU)) * XGMI_LINK_GBPS


def p50(latencies: Iterable[float]) -> float:
    return statistics.median(list(latencies))
