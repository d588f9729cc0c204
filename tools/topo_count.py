#!/usr/bin/env python3
"""Search-space size of FlexTree topologies: H(n), the number of ordered factorizations of n.

Reference: topo_count/factor_count.py:1-15 (exponential recursion, prints H(0)).
Here memoised; prints H(n) for the arguments (default 1..16) and cross-checks the
native planner's count.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from allreduce_over_mpi_amd.utils.topology import get_factor_count  # noqa: E402

if __name__ == "__main__":
    ns = [int(a) for a in sys.argv[1:]] or list(range(1, 17))
    try:
        from allreduce_over_mpi_amd import _native as nv

        native = nv.count_factorizations
    except Exception:  # library not built: pure Python only
        native = None
    for n in ns:
        h = get_factor_count(n)
        extra = "" if native is None else ("" if native(n) == h else f"  (native {native(n)} MISMATCH)")
        print(f"{n}\t{h}{extra}")
