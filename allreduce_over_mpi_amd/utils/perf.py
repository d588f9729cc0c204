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


def recommend_bucket_bytes(cost_us, efficiency: float = 0.9, lo: int = 1 << 20, hi: int = 1 << 30,
                           quantum: int = 1 << 20) -> int:
    """Smallest gradient-bucket size (a multiple of ``quantum``, within [lo, hi]) whose predicted allreduce
    bandwidth ``bytes / cost_us(bytes)`` reaches ``efficiency`` of the bandwidth at ``hi``.

    Bucket size trades overlap (small buckets start reducing early in the backward pass) against the fixed
    launch and hand-off cost of every call. On an MI355X node the knee is set by xGMI, not by the
    interconnect a default was tuned for (DDP's 25 MiB): ``cost_us`` is the calibrated selector's price
    (``Communicator.predict_us("auto", b)``), so the answer follows the links this job actually runs on.
    Bisection over multiples of ``quantum``; assumes bandwidth grows with the size (as the model's does)."""
    if not 0 < efficiency < 1 or lo < 1 or hi < lo:
        raise ValueError("need 0 < efficiency < 1 and 1 <= lo <= hi")
    target = efficiency * hi / cost_us(float(hi))
    a, b = max(1, lo // quantum), max(1, hi // quantum)  # in quanta: answer in (a - 1, b]
    if (a * quantum) / cost_us(float(a * quantum)) >= target:
        return a * quantum
    while b - a > 1:
        m = (a + b) // 2
        if (m * quantum) / cost_us(float(m * quantum)) >= target:
            b = m
        else:
            a = m
    return b * quantum
