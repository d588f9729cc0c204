"""Connect-time readiness logic on the CPU (csrc/include/flexar/readiness.hpp).

The GPU half (the probe and the exact self-test on real peers) is in tests/test_gpu_ipc.py and
tests/test_gpu_multidevice.py; here the downgrade chain, the link-count rule and the planner's
cross-rank staging agreement are checked with injected inputs.
"""
import re

import pytest

from allreduce_over_mpi_amd import _native as nv


@pytest.mark.parametrize("spec,failed,expect", [
    ("flat+pull", [], "tree:8+pull"),
    ("flat+pull", ["fence"], "tree:8+pull+wt"),
    ("flat+pull+nts", ["fence"], "tree:8+pull+wt"),          # +nts is the fence family too
    ("ring:2", ["fence"], "ring:2+wt"),
    ("rhd+pull", ["fence"], "tree:2,2,2+pull+wt"),
    ("flat+pull", ["fence", "wt"], "dma"),                   # executor unusable: copy engines
    ("ll", ["ll"], "oneshot"),
    ("ll", ["ll", "fence"], "oneshot+wt"),
    ("dma", ["dma"], "tree:8+pull"),
    ("dma", ["dma", "fence"], "tree:8+pull+wt"),
    ("flat+pull+wt", ["wt"], "dma"),
])
def test_downgrade_chain(spec, failed, expect):
    assert nv.downgrade_spec(spec, 8, failed) == expect


def test_downgrade_without_dma_and_exhausted():
    # RS/AG/broadcast cannot switch to the copy-engine allreduce
    with pytest.raises(nv.FlexarError) as e:
        nv.downgrade_spec("flat+pull", 8, ["fence", "wt"], allow_dma=False)
    assert e.value.rc == 2 and "fence,wt" in str(e.value)
    with pytest.raises(nv.FlexarError):
        nv.downgrade_spec("ll", 8, ["fence", "wt", "ll", "dma"])
    # a mask with nothing failed leaves every spec alone
    for s in ("ring", "tree:2,4+pull", "oneshot", "ll", "dma"):
        assert nv.downgrade_spec(s, 8, 0) == nv.downgrade_spec(s, 8, [])


def test_direct_links_rule():
    # fully connected 8-GPU xGMI node: 7 direct links for every rank
    cls = ["xgmi"] * 8
    hops = [1] * 8
    cls[3] = "same-device"  # the rank itself (ignored)
    assert nv.direct_links(cls, hops, 3) == 7
    # two-hop peers are not direct links; PCIe peers neither
    assert nv.direct_links(["xgmi", "xgmi", "xgmi", "pcie"], [1, 2, 1, 1], 0) == 1
    # ranks sharing one GPU: no link at all -> at least one (the shared HBM)
    assert nv.direct_links(["same-device"] * 4, [0] * 4, 1) == 1
    # peers this process cannot see (HIP_VISIBLE_DEVICES) are assumed direct
    assert nv.direct_links(["unknown"] * 4, [0] * 4, 2) == 3


def _staging(spec, rank, n, count):
    dump = nv.plan_dump(spec, rank, n, count)
    return int(re.search(r"staging (\d+) elems/parity", dump).group(1))


@pytest.mark.parametrize("n,spec", [(7, "tree:2,3"), (7, "tree:3,2+pull"), (5, "tree:2,2"), (7, "tree:2,2+push")])
def test_lonely_ranks_report_the_tree_staging(n, spec):
    """every rank sizes its pieces from its own staging figure, so lonely ranks must
    report the tree ranks' figure or the ranks split a call into different piece counts."""
    for count in (35, 1 << 20, (57 << 20) // 4):
        figs = {_staging(spec, r, n, count) for r in range(n)}
        assert len(figs) == 1, (spec, count, figs)


def test_lonely_split_call_in_simulator():
    """A lonely-tree allreduce still sums correctly when every rank uses the common staging size."""
    import numpy as np

    rng = np.random.default_rng(3)
    ins = [rng.integers(-50, 50, 4099).astype(np.int32) for _ in range(7)]
    outs = nv.simulate("tree:2,3+pull", ins, grid=2, ncalls=3)
    want = np.sum(ins, axis=0)
    for o in outs:
        np.testing.assert_array_equal(o, want)
