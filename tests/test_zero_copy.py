"""Zero-copy flat allreduce over registered buffers ("+zc", planner.hpp build_flat_zc) on the CPU simulator.

The program reads every peer's IN (reduce-scatter) and OUT (all-gather) directly - the device executor
does the same through IPC-mapped registered buffers (comm.hip zc_bind, flexar_reg_*). Checked here:
exact sums for every rank count including uneven tails and in-place calls, determinism across ranks,
the program shape (no staging, three hand-offs), and that the spec is refused where it cannot run.
"""
import numpy as np
import pytest

from allreduce_over_mpi_amd import _native as nv


@pytest.mark.parametrize("n", [2, 3, 4, 7, 8, 12, 16])
@pytest.mark.parametrize("count", [1, 35, 4099, 10007])
@pytest.mark.parametrize("spec", ["flat+zc", "flat+zc+wt", "flat+zc+nts", "flat+zc+push", "flat+zc+push+wt",
                                  "flat+zc+put", "flat+zc+put+wt"])
def test_zero_copy_exact_sum(n, count, spec):
    ins = [np.random.default_rng(7 * r + count).integers(-99, 99, count).astype(np.int32) for r in range(n)]
    want = np.sum(ins, axis=0)
    for o in nv.simulate(spec, ins, ncalls=3, grid=3):
        np.testing.assert_array_equal(o, want)


@pytest.mark.parametrize("n", [2, 4, 8, 11])
@pytest.mark.parametrize("spec", ["flat+zc", "flat+zc+push", "flat+zc+put"])
def test_zero_copy_in_place(n, spec):
    # IN == OUT: block k of a rank's IN is read only by its owner k, which overwrites it (push) or lets it
    # be overwritten (pull) only afterwards
    ins = [np.random.default_rng(r).integers(-50, 50, 5003).astype(np.int32) for r in range(n)]
    want = np.sum(ins, axis=0)
    for o in nv.simulate(spec, ins, ncalls=4, grid=4, in_place=True):
        np.testing.assert_array_equal(o, want)


def test_zero_copy_float_is_rank_order_deterministic():
    n = 8
    ins = [np.random.default_rng(r).standard_normal(9001).astype(np.float32) * (r + 1) for r in range(n)]
    outs = nv.simulate("flat+zc", ins, grid=2, op="avg")
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])  # the owner of each block sums in rank order; others copy it
    np.testing.assert_allclose(outs[0], np.mean(np.stack(ins).astype(np.float64), axis=0), rtol=1e-5, atol=1e-5)
    # every zero-copy form sums in the same rank order: identical bits
    for spec in ("flat+zc+push", "flat+zc+put"):
        for o in nv.simulate(spec, ins, grid=2, op="avg"):
            assert np.array_equal(o, outs[0]), spec


def test_zero_copy_program_shape():
    d = nv.plan_dump("flat+zc", 1, 4, 4096, "float32")
    assert "staging 0 elems" in d and "3 flag slots" in d
    assert "IN@0" in d and "OUT@2" in d  # peer buffers are addressed directly
    assert "STG" not in d
    # push: one reduction straight into every rank's OUT, two hand-offs
    d = nv.plan_dump("flat+zc+push", 1, 4, 4096, "float32")
    assert "2 flag slots" in d and d.count("XFER") == 1 and "STG" not in d
    # put: remote writes only - three pushes into the owners' staging, one reduction into every OUT; no
    # peer IN is addressed (only the outputs need registering)
    d = nv.plan_dump("flat+zc+put", 1, 4, 4096, "float32")
    assert "2 flag slots" in d and d.count("XFER") == 4, d
    assert "OUT@0" in d and "OUT@2" in d and "IN@0" not in d and "IN@2" not in d, d


def test_zero_copy_refused_outside_flat():
    ins = [np.zeros(64, np.int32) for _ in range(4)]
    for spec in ("ring+zc", "rhd+zc", "tree:2,2+zc", "tree:2,2+zc+put"):
        with pytest.raises(nv.FlexarError):
            nv.simulate(spec, ins)


@pytest.mark.parametrize("n", [2, 3, 4, 8, 12])
def test_zero_copy_collectives(n):
    """Reduce-scatter (pull), all-gather (push), all-to-all (push) and broadcast (root push) straight over
    the peers' registered buffers."""
    m = 1001
    ins = [np.random.default_rng(r).integers(-50, 50, n * m).astype(np.int32) for r in range(n)]
    tot = np.sum(ins, axis=0)
    rs = nv.simulate_coll("reduce_scatter", "flat+zc", ins, m, dtype="int32", ncalls=3)
    for r in range(n):
        np.testing.assert_array_equal(rs[r], tot[r * m:(r + 1) * m])
    ag_in = [np.random.default_rng(10 + r).integers(-50, 50, m).astype(np.int32) for r in range(n)]
    for o in nv.simulate_coll("all_gather", "flat+zc", ag_in, m, dtype="int32", ncalls=3):
        np.testing.assert_array_equal(o, np.concatenate(ag_in))
    a2a = nv.simulate_coll("all_to_all", "flat+zc", ins, m, dtype="int32", ncalls=3)
    for r in range(n):
        np.testing.assert_array_equal(a2a[r], np.concatenate([ins[q][r * m:(r + 1) * m] for q in range(n)]))
    data = np.arange(5003, dtype=np.float32)
    for root in (0, n - 1):
        for o in nv.simulate_bcast("flat+zc", data, n, root=root):
            np.testing.assert_array_equal(o, data)


def test_zero_copy_collectives_refuse_ring():
    ins = [np.zeros(4 * 64, np.int32) for _ in range(4)]
    with pytest.raises(nv.FlexarError):
        nv.simulate_coll("reduce_scatter", "ring+zc", ins, 64, dtype="int32")


def test_zero_copy_policy():
    """The automatic zero-copy switch (csrc/include/flexar/zc_policy.hpp, applied by comm.hip per call)."""
    big, small = float(1 << 28), 8192.0
    # registered buffers, automatic choice: the flat schedule always switches, keeping its protocol
    assert nv.zc_decide("flat+pull", 8, big) == (1, "tree:8+push+zc")
    assert nv.zc_decide("flat+pull+wt", 8, big) == (1, "tree:8+push+wt+zc")
    # another model choice only when the model prices the push form lower: large oneshot yes, small LL no
    assert nv.zc_decide("oneshot", 2, big)[0] == 1
    assert nv.zc_decide("ll", 8, small) == (0, "ll")
    # a tune table's measured non-flat choice is kept; its flat choice still switches
    assert nv.zc_decide("ring", 8, big, have_tune=True) == (0, "ring")
    assert nv.zc_decide("flat+pull", 8, big, have_tune=True)[0] == 1
    # never: unregistered, a named spec, FLEXAR_ZC_AUTO=0, one rank, copy engines, typed / message transport
    assert nv.zc_decide("flat+pull", 8, big, registered=False)[0] == 0
    assert nv.zc_decide("flat+pull", 8, big, named=True, auto=False)[0] == 0
    assert nv.zc_decide("flat+pull", 8, big, zc_auto=False)[0] == 0
    assert nv.zc_decide("flat+pull", 1, big)[0] == 0
    assert nv.zc_decide("dma", 8, big)[0] == 0
    assert nv.zc_decide("flat+rccl", 8, big)[0] == 0
    # a protocol family that failed the connect-time self-test is never picked by the switch
    fence = nv.FAMILIES["fence"]
    assert nv.zc_decide("flat+pull", 8, big, disabled=fence)[0] == 0
    assert nv.zc_decide("flat+pull+wt", 8, big, disabled=fence)[0] == 1
    # a zero-copy choice nobody named (tune table, default spec) falls back for unregistered buffers; a named
    # one stays (and is refused at the call with an error)
    assert nv.zc_decide("flat+zc+push", 8, big, registered=False, auto=False) == (-1, "tree:8+push")
    assert nv.zc_decide("flat+zc+push", 8, big, registered=False, named=True, auto=False) == (0, "tree:8+push+zc")
    assert nv.zc_decide("flat+zc+put", 8, big, registered=False, auto=False) == (-1, "tree:8+push")
    assert nv.zc_decide("flat+zc+put", 8, big, auto=False) == (0, "tree:8+zc+put")
