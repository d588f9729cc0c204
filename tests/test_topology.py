"""Topology parsing, enumeration and the cost models (host only).

Reference behaviour pinned from SURVEY.md §2.5/§4.2 (verified by running the
reference): FT_TOPO unset -> flat {N}; any 1 -> ring; product != N -> error;
'2,2,2,' failed in the reference (defect D4) and is accepted here.
"""
import pytest


def test_ft_topo_reference_rules(nv):
    assert nv.parse_ft_topo(None, 8) == "tree:8"
    assert nv.parse_ft_topo("", 8) == "tree:8"
    assert nv.parse_ft_topo("2,2,2", 8) == "tree:2,2,2"
    assert nv.parse_ft_topo("2 2 2", 8) == "tree:2,2,2"
    assert nv.parse_ft_topo("2, 2,2", 8) == "tree:2,2,2"
    assert nv.parse_ft_topo("2,4", 8) == "tree:2,4"
    assert nv.parse_ft_topo("4,1,2", 8) == "ring"      # any 1 -> ring (mpi_mod.hpp:907-910)
    assert nv.parse_ft_topo("1", 5) == "ring"
    assert nv.parse_ft_topo("2,3", 6) == "tree:2,3"


def test_ft_topo_d4_fixed(nv):
    # reference: trailing separator re-pushes the last token -> 'invalid FT_TOPO' exit(1)
    assert nv.parse_ft_topo("2,2,2,", 8) == "tree:2,2,2"
    assert nv.parse_ft_topo(",2,,4,", 8) == "tree:2,4"


@pytest.mark.parametrize("bad,n", [("2,3", 8), ("0", 8), ("3", 8), ("2,x", 8), ("-2,-4", 8)])
def test_ft_topo_invalid(nv, bad, n):
    with pytest.raises(nv.FlexarError):
        nv.parse_ft_topo(bad, n)


def test_factor_count_matches_reference_tool(nv):
    from allreduce_over_mpi_amd.utils.topology import get_factor_count

    # reference topo_count/factor_count.py: recursive H(n)
    def ref(num):
        if num == 0:
            return 0
        if num == 1:
            return 1
        return sum(ref(num // i) for i in range(2, num + 1) if num % i == 0)

    for n in list(range(0, 65)) + [96, 128, 340]:
        assert nv.count_factorizations(n) == ref(n) == get_factor_count(n), n
    # survey: 5 / 9 / 45 reference candidates for N = 8 / 16 / 340 (= H(N) + 1 with [N] duplicated)
    assert [nv.count_factorizations(n) + 1 for n in (8, 16, 340)] == [5, 9, 45]


def test_enumerate_plans(nv):
    p8 = nv.enumerate_plans(8)
    assert "tree:8" in p8 and "tree:2,2,2" in p8 and "tree:2,4" in p8 and "tree:4,2" in p8
    assert "ring" in p8 and "ring:4" in p8 and "oneshot" in p8 and "ll" in p8
    trees = [p for p in p8 if p.startswith("tree:") and p.count(":") == 1]
    assert len(trees) == nv.count_factorizations(8)
    # every multi-stage tree again on N - 1 link-balanced channels (planner.hpp build_tree_channels)
    assert sorted(p for p in p8 if p.count(":") == 2) == ["tree:2,2,2:7", "tree:2,4:7", "tree:4,2:7"]
    p7 = nv.enumerate_plans(7)  # prime: flat tree + rings
    assert "tree:7" in p7 and "ring:6" in p7
    assert nv.enumerate_plans(1) == []


def test_legacy_cost_model_worked_example(nv):
    # N = 8, s = 100, 2*2*2 = 3 x 0.008 + 0.105 + 0.595 = 0.724
    assert nv.legacy_cost([2, 2, 2], 8, 100) == pytest.approx(0.724, abs=1e-9)
    # reference picks '1*8' (= flat) for N <= 9 at s = 100: flat must be the argmin among trees
    from allreduce_over_mpi_amd.utils.topology import legacy_best

    assert legacy_best(8, 100)[0] == [8]
    assert legacy_best(16, 100)[0] == [2, 8]   # survey table: N=16, s=100 -> 2*8
    assert legacy_best(64, 100)[0] == [8, 8]   # survey table: N=64, s=100 -> 8*8


def test_xgmi_selector_prefers_all_links(nv):
    # On a fully connected 8-GPU mesh the flat stage drives 7 links; it must beat 1-link plans for big buffers.
    big = 256 << 20
    assert nv.model_cost_us("flat", 8, big) < nv.model_cost_us("ring", 8, big)
    assert nv.model_cost_us("flat", 8, big) < nv.model_cost_us("rhd", 8, big)
    assert nv.select_plan(8, big).startswith("tree:8")
    # tiny buffers: a single stage (oneshot) beats 2(N-1) ring hops
    assert nv.model_cost_us("oneshot", 8, 4096) < nv.model_cost_us("ring", 8, 4096)
    assert nv.select_plan(8, 4096) in ("ll", "oneshot")
    assert nv.model_cost_us("ll", 8, 4096) < nv.model_cost_us("oneshot", 8, 4096)


def test_algo_spec_errors(nv):
    with pytest.raises(nv.FlexarError):
        nv.model_cost_us("rhd", 6, 1e6)        # not a power of two
    with pytest.raises(nv.FlexarError):
        nv.model_cost_us("tree:3", 8, 1e6)     # product < N/2
    with pytest.raises(nv.FlexarError):
        nv.model_cost_us("tree:4,4", 8, 1e6)   # product > N
    assert nv.model_cost_us("tree:2,2", 8, 1e6) > 0  # 4 lonely ranks folded into 4 partners
    with pytest.raises(nv.FlexarError):
        nv.model_cost_us("bogus", 8, 1e6)


def test_protocol_modifiers(nv):
    # "+nts" / "+wt" change only the executor's memory protocol, never the schedule
    for spec in ("flat+wt", "flat+push+wt", "ring:2+wt", "oneshot+wt", "flat+nts+wt"):
        assert nv.model_cost_us(spec, 8, 1e6) > 0
        base = spec.replace("+wt", "").replace("+nts", "")
        body = lambda sp: nv.plan_dump(sp, 1, 8, 4096).split("\n", 1)[1]  # noqa: E731 (header names the spec)
        assert body(spec) == body(base)
    with pytest.raises(nv.FlexarError):
        nv.model_cost_us("flat+wtx", 8, 1e6)


def test_dma_spec(nv):
    # copy-engine allreduce: device-only engine, host programs run the same flat exchange
    assert nv.model_cost_us("dma", 8, 256e6) > 0
    assert nv.model_cost_us("dma", 8, 4096) > nv.model_cost_us("ll", 8, 4096)
    body = lambda sp: nv.plan_dump(sp, 2, 8, 1000).split("\n", 1)[1]  # noqa: E731
    assert body("dma") == body("flat+pull")


def _remote_elems(dump, rank):
    """Elements a rank's program moves over links: every XFER operand in another rank's staging."""
    import re

    total = 0
    for line in dump.splitlines():
        m = re.match(r"\s+XFER len=(\d+) \[(.*)\] -> \[(.*)\]", line)
        if not m:
            continue
        locs = m.group(2).split(" + ") + m.group(3).split(", ")
        remote = sum(1 for loc in locs if loc.startswith("STG@") and int(loc[4:].split(":")[0]) != rank)
        total += int(m.group(1)) * remote
    return total


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 8, 12, 16])
def test_plans_move_bandwidth_optimal_bytes(nv, n):
    """every tree/ring/flat schedule moves 2(N-1)/N * S per rank (the reference's
    'key structural fact'); oneshot moves (N-1) * S. Checked on the compiled programs of every rank."""
    count = 16384 * n  # large enough that 16-element block rounding stays < 1 % (ring:7 splits 7 ways)
    specs = [p for p in nv.enumerate_plans(n) if p.startswith(("tree:", "ring"))]
    specs = [s for s in specs if not s.startswith("tree:") or
             __import__("math").prod(int(w) for w in s[5:].split(":")[0].split(",")) == n]  # lonely trees fold extra data
    specs += [s + "+push" for s in specs if s.startswith("tree:")] + ["flat", "oneshot", "flat+bidir"]
    for spec in specs:
        if spec.split("+")[0].count(":") == 2:  # N - 1 channels: slices of whole aligned blocks
            count = n * (n - 1) * 4096
        else:
            count = 16384 * n
        want = (n - 1) * count if spec == "oneshot" else 2 * (n - 1) * count / n
        for r in range(n):
            got = _remote_elems(nv.plan_dump(spec, r, n, count), r)
            assert abs(got - want) <= 0.01 * want, (spec, n, r, got, want)


def test_selection_table_matches_selector():
    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.utils.topology import selection_table

    rows = selection_table(8, [4096, 1 << 20, 256 << 20])
    assert [r[1] for r in rows] == [nv.select_plan(8, b) for b in (4096, 1 << 20, 256 << 20)]
    assert rows[0][2] < rows[1][2] < rows[2][2]


def _ordered_factorizations(n):
    if n == 1:
        return [[]]
    return [[d] + rest for d in range(2, n + 1) if n % d == 0 for rest in _ordered_factorizations(n // d)]


@pytest.mark.parametrize("lo,hi", [(2, 16), (17, 32), (33, 48), (49, 64)])
def test_every_ordered_factorization_up_to_64(nv, lo, hi):
    """the plan generator's invariants for EVERY ordered factorization of every N <= 64 (the
    reference's whole FT_TOPO space: H(N) trees per N, plus the ring). Every rank ends with the exact sum
    (uneven tail blocks: count is not a multiple of N), and every rank's program moves the
    bandwidth-optimal 2 (N - 1) / N of the buffer over the links. The widths come from an independent
    enumeration and are checked against the native one (count = H(N))."""
    import math

    import numpy as np

    for n in range(lo, hi + 1):
        facts = _ordered_factorizations(n)
        assert len(facts) == nv.count_factorizations(n), n
        specs = ["tree:" + ",".join(map(str, f)) for f in facts] + ["ring"]
        count = 7 * n + 3  # uneven: the last block is short
        ins = [np.arange(count, dtype=np.int64) * (r + 1) + r for r in range(n)]
        want = np.sum(ins, axis=0)
        big = 4096 * n
        for spec in specs:
            for o in nv.simulate(spec, ins, ncalls=2):
                assert np.array_equal(o, want), (spec, n)
            if n <= 32 or spec.count(",") <= 1:  # the byte count over every rank's dump, sampled above 32
                for r in (0, n - 1):
                    got = _remote_elems(nv.plan_dump(spec, r, n, big), r)
                    assert abs(got - 2 * (n - 1) * big / n) <= 0.01 * big, (spec, n, r, got)
        assert math.prod(facts[0]) == n
