"""Topology helpers on top of csrc/include/flexar/topology.hpp + cost_model.hpp (through ``_native``).

* ``get_factor_count`` - the size of the FlexTree search space H(n), the number of ordered factorizations
  of n (reference ``topo_count/factor_count.py:1-15``, an exponential recursion): a divisor DP here,
  checked against the native ``count_factorizations`` in tests/test_topology.py.
* ``legacy_best`` - the reference cost model's argmin over ordered factorizations (CostModel.h:82-119).
* ``selection_table`` - the runtime selector's choice and predicted time per buffer size (what
  ``tools/flexar_plan select`` prints), for reports and notebooks.
"""
from __future__ import annotations

from functools import lru_cache

from .. import _native as nv


@lru_cache(maxsize=None)
def get_factor_count(num: int) -> int:
    """H(num): ordered factorizations of num into factors >= 2 (H(1) = 1, H(n <= 0) = 0)."""
    if num <= 0:
        return 0
    h = [0] * (num + 1)
    h[1] = 1
    for m in range(2, num + 1):
        h[m] = sum(h[m // f] for f in range(2, m + 1) if m % f == 0)
    return h[num]


def legacy_best(nranks: int, chunk: float = 100.0):
    """The reference cost model's argmin over ordered factorizations: (widths, cost)."""
    best = None
    for p in nv.enumerate_plans(nranks):
        if not p.startswith("tree:") or p.count(":") > 1:  # a channelled copy has the same widths
            continue
        w = [int(x) for x in p[5:].split("+")[0].split(",")]
        c = nv.legacy_cost(w, nranks, chunk)
        if best is None or c < best[1]:
            best = (w, c)
    return best


def selection_table(nranks: int, sizes=None):
    """[(bytes, spec, predicted_us)] of the runtime selector (FLEXAR_MODEL / defaults) per buffer size."""
    sizes = sizes or [4096 << (2 * k) for k in range(11)]
    rows = []
    for b in sizes:
        spec = nv.select_plan(nranks, float(b))
        rows.append((b, spec, nv.model_cost_us(spec, nranks, float(b))))
    return rows
