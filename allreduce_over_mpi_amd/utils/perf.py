"""Bandwidth bookkeeping (rccl-tests convention).

algbw = bytes / time;  busbw = algbw * 2 (N - 1) / N  (allreduce).
busbw is the per-rank link-level rate: constant in N for a bandwidth-optimal
algorithm, so it is the number compared across N and against RCCL.
"""
from __future__ import annotations


def algbw_gbps(nbytes: float, seconds: float) -> float:
    return nbytes / seconds / 1e9 if seconds > 0 else 0.0


def busbw_factor(nranks: int) -> float:
    return 2.0 * (nranks - 1) / nranks if nranks > 0 else 0.0


def busbw_gbps(nbytes: float, seconds: float, nranks: int) -> float:
    return algbw_gbps(nbytes, seconds) * busbw_factor(nranks)


def human_bytes(n: float) -> str:
    for unit in ("B", "KiB", "MiB", "GiB", "TiB"):
        if n < 1024 or unit == "TiB":
            return f"{n:.0f}{unit}" if unit == "B" else f"{n:.1f}{unit}"
        n /= 1024.0
    return str(n)
