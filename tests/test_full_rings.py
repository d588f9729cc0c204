"""Multi-channel rings over the full xGMI mesh (csrc/include/flexar/topology.hpp hamiltonian_decomposition).

The circulant rings r -> r + d stop at 4 channels on 8 ranks (only odd d are Hamiltonian), i.e. 4 of a
GPU's 7 xGMI links. The complete digraph splits into N - 1 arc-disjoint directed Hamiltonian cycles for
every N except 4 and 6, so `ring:7` at N = 8 drives every outgoing link of every GPU. These tests pin the
decomposition (Hamiltonian, arc-disjoint, identical on every call), the planner's use of it (exact sums in
the CPU simulator, busiest-link bytes equal to flat's), and that rings that fit the circulants keep their
orders. Reference counterpart: the single ring of allreduce_over_mpi/mpi_mod.hpp:1114-1160 (one ring,
rank order, MPI point-to-point).
"""
import numpy as np
import pytest

from allreduce_over_mpi_amd import _native as nv


def _arcs(order):
    n = len(order)
    return {(order[i], order[(i + 1) % n]) for i in range(n)}


@pytest.mark.parametrize("n", list(range(2, 17)))
def test_ring_channels_are_hamiltonian_and_arc_disjoint(n):
    _, maxc = nv.ring_order(n, 0, 1)
    slot_cap = 126 // (2 * (n - 1))
    circ = sum(1 for d in range(1, n) if np.gcd(d, n) == 1)
    full = 0 if n in (4, 6) else n - 1
    assert maxc == max(1, min(max(circ, full), slot_cap)), (n, maxc)
    for C in range(1, maxc + 1):
        seen = set()
        for c in range(C):
            o, _ = nv.ring_order(n, c, C)
            assert sorted(o) == list(range(n)), (n, C, c, o)
            a = _arcs(o)
            assert not (a & seen), ("arcs reused", n, C, c)
            seen |= a
        assert nv.ring_order(n, C - 1, C)[0] == nv.ring_order(n, C - 1, C)[0]  # deterministic


def test_eight_ranks_use_every_link():
    n, C = 8, 7
    arcs = set()
    for c in range(C):
        arcs |= _arcs(nv.ring_order(n, c, C)[0])
    assert arcs == {(a, b) for a in range(n) for b in range(n) if a != b}


def test_circulant_orders_kept_where_they_fit():
    for n, C in ((8, 2), (8, 4), (5, 4), (7, 6)):
        for c in range(C):
            d = [k for k in range(1, n) if np.gcd(k, n) == 1][c]
            assert nv.ring_order(n, c, C)[0] == [(p * d) % n for p in range(n)]


@pytest.mark.parametrize("n,spec", [(8, "ring:7"), (8, "ring:5"), (9, "ring:7"), (5, "ring:4")])
def test_full_mesh_ring_is_exact(n, spec):
    rng = np.random.default_rng(n)
    xs = [rng.integers(-1000, 1000, size=4099).astype(np.float32) for _ in range(n)]
    want = np.sum(np.stack(xs).astype(np.float64), axis=0)
    outs = nv.simulate(spec, xs, grid=2 * int(spec.split(":")[1]))  # grid: a multiple of the channels
    for o in outs:
        assert np.array_equal(np.asarray(o, dtype=np.float64), want), spec


def test_full_mesh_ring_prices_like_flat_on_links():
    count = 16 << 20
    r7 = nv.program_cost("ring:7", 0, 8, count, "float32", links=7)
    r4 = nv.program_cost("ring:4", 0, 8, count, "float32", links=7)
    flat = nv.program_cost("flat+pull", 0, 8, count, "float32", links=7)
    assert r7["link_time_bytes"] == pytest.approx(flat["link_time_bytes"], rel=1e-3)
    assert r7["link_time_bytes"] == pytest.approx(r4["link_time_bytes"] * 4 / 7, rel=1e-3)
    assert "ring:7" in nv.enumerate_plans(8)
