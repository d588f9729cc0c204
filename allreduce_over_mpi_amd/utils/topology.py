"""Topology helpers (Python face of csrc/include/flexar/topology.hpp + cost_model.hpp).

* ``get_factor_count`` — reference ``topo_count/factor_count.py:1-15`` (number of
  ordered factorizations H(n), i.e. the size of the FlexTree search space), here
  memoised instead of exponential.
* ``parse_ft_topo`` / ``enumerate_plans`` / ``select_plan`` / ``legacy_cost`` call
  the native implementations so Python and the runtime can never disagree.
"""
from __future__ import annotations

from functools import lru_cache

from .. import _native as nv


@lru_cache(maxsize=None)
def get_factor_count(num: int) -> int:
    if num <= 0:
        return 0
    if num == 1:
        return 1
    return sum(get_factor_count(num // i) for i in range(2, num + 1) if num % i == 0)


def parse_ft_topo(ft_topo, nranks: int) -> str:
    return nv.parse_ft_topo(ft_topo, nranks)


def enumerate_plans(nranks: int):
    return nv.enumerate_plans(nranks)


def select_plan(nranks: int, nbytes: float) -> str:
    return nv.select_plan(nranks, nbytes)


def model_cost_us(spec: str, nranks: int, nbytes: float) -> float:
    return nv.model_cost_us(spec, nranks, nbytes)


def legacy_cost(widths, nranks: int, chunk: float = 100.0) -> float:
    return nv.legacy_cost(widths, nranks, chunk)


def legacy_best(nranks: int, chunk: float = 100.0):
    """The reference cost model's argmin over ordered factorizations (CostModel.h:82-119)."""
    best = None
    for p in nv.enumerate_plans(nranks):
        if not p.startswith("tree:"):
            continue
        w = [int(x) for x in p[5:].split("+")[0].split(",")]
        c = nv.legacy_cost(w, nranks, chunk)
        if best is None or c < best[1]:
            best = (w, c)
    return best
