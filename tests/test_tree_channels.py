"""Multi-channel, link-balanced FlexTree schedules ("rhd:C", "tree:a,b:C").

The reference's mixed-radix tree puts a rank in one group of w_s members per stage
(/root/reference/allreduce_over_mpi/mpi_mod.hpp:147-214 Send_Ops / Recv_Ops), so on a fully
connected xGMI mesh stage s of one tree drives w_s - 1 of a GPU's N - 1 links (RHD: one). C channels
run the same tree over disjoint slices with relabelled ranks (planner.hpp build_tree_channels,
topology.hpp tree_channel_labels: a Singer cycle of GF(2^k) for power-of-two N, a deterministic greedy
search otherwise) so that every stage covers the links evenly. These CPU tests pin exactness (the
simulator runs the exact op programs of the gfx950 executor), the link balance read off the compiled
programs, and the cost model's pricing.
"""
import re

import numpy as np
import pytest

from test_simulator import channels_of

CASES = [(2, "rhd:3"), (4, "rhd:3"), (4, "rhd:3+push"), (4, "tree:2,2:3+nofuse"), (8, "rhd:7"), (8, "rhd:7+pull"),
         (8, "rhd:7+push+nofuse"), (8, "tree:4,2:7+pull"), (8, "tree:2,4:7+push"), (8, "rhd:3"), (8, "rhd:14"),
         (6, "tree:2,3:5"), (6, "tree:3,2:5+push"), (12, "tree:3,4:11+pull"), (16, "rhd:15+pull"),
         (16, "tree:4,4:15")]


@pytest.mark.parametrize("n,spec", CASES)
def test_exact_with_tails_and_in_place(nv, n, spec):
    """Integer sums (exact) for sizes with uneven tails, including sizes smaller than the channel count
    (empty channels still hand off), out of place and in place, over consecutive calls (both parities)."""
    C = channels_of(spec)
    for size in (1, 5, 35, 1001, 65539):
        ins = [np.random.default_rng(13 * r + size).integers(-999, 999, size).astype(np.int64) for r in range(n)]
        want = np.sum(np.stack(ins), 0)
        for in_place in (False, True):
            for r, o in enumerate(nv.simulate(spec, ins, grid=2 * C, ncalls=3, in_place=in_place)):
                np.testing.assert_array_equal(o, want, err_msg=f"{spec} n={n} size={size} r={r} ip={in_place}")


@pytest.mark.parametrize("spec", ["rhd:7+pull+f32", "rhd:7+pull+rw", "tree:4,2:7+f32"])
def test_typed_partials_bf16(nv, spec):
    """bf16 with fp32 partials (one rounding: bit-equal to the fp32 sum rounded once) and per-hop rounding
    (+rw: within 3 roundings) on the channelled trees."""
    import torch

    n = 8
    xs = [np.random.default_rng(r).standard_normal(9001).astype(np.float32) for r in range(n)]
    bits = [torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16) for x in xs]
    vals = [torch.from_numpy(b.view(np.int16)).view(torch.bfloat16).double().numpy() for b in bits]
    exact = np.sum(np.stack(vals), 0)
    outs = nv.simulate_typed(spec, bits, "bfloat16", grid=14, ncalls=2)
    got = [torch.from_numpy(o.view(np.int16)).view(torch.bfloat16).double().numpy() for o in outs]
    for g in got[1:]:
        np.testing.assert_array_equal(g, got[0])  # every rank holds the owner's bits
    if spec.endswith("+f32") or "+f32" in spec:
        # one rounding of an fp32 partial sum: within 1 bf16 ulp of the exact sum
        np.testing.assert_allclose(got[0], exact, rtol=2 ** -7, atol=1e-6)
    else:
        np.testing.assert_allclose(got[0], exact, rtol=3 * 2 ** -7, atol=3 * 2 ** -7 * np.abs(np.stack(vals)).sum(0).max())


def _stage_peers(dump):
    """channel -> list of (slot, sorted peers) of its SIGNAL ops, in program order."""
    out, ch = {}, None
    for line in dump.splitlines():
        m = re.match(r"channel (\d+):", line)
        if m:
            ch = int(m.group(1))
            out[ch] = []
            continue
        m = re.match(r"\s+SIGNAL slot=(\d+) peers=([\d,]+)", line)
        if m:
            out[ch].append((int(m.group(1)), sorted(int(p) for p in m.group(2).split(","))))
    return out


def test_rhd7_uses_every_link_in_every_stage(nv):
    """rhd:7 at N = 8: in each of the 3 reduce-scatter stages, the 7 channels pair every rank with 7
    distinct partners - all of its xGMI links - where single-channel RHD uses one."""
    n = 8
    for rank in range(n):
        peers = _stage_peers(nv.plan_dump("rhd:7+pull", rank, n, 1 << 20))
        assert len(peers) == 7
        for stage in range(3):
            partners = [peers[c][stage][1] for c in range(7)]
            assert all(len(p) == 1 for p in partners)
            assert sorted(p[0] for p in partners) == sorted(set(range(n)) - {rank}), (rank, stage, partners)
            # each channel has its own flag slots
            assert [peers[c][stage][0] for c in range(7)] == [c * 6 + stage for c in range(7)]
        # channel 0 is the single-channel tree itself
        assert [p for _, p in peers[0]] == [p for _, p in _stage_peers(nv.plan_dump("rhd+pull", rank, n, 1 << 20))[0]]


@pytest.mark.parametrize("n,spec", [(8, "tree:4,2:7"), (8, "tree:2,4:7"), (4, "rhd:3"), (16, "rhd:15"),
                                    (16, "tree:4,4:15"), (16, "tree:2,8:15")])
def test_power_of_two_stages_balanced(nv, n, spec):
    """Singer-cycle relabelling: over C = N - 1 channels each stage uses every link equally often."""
    w = [int(x) for x in spec.split(":")[1].split(",")] if spec.startswith("tree") else [2] * (n.bit_length() - 1)
    for rank in (0, n - 1):
        peers = _stage_peers(nv.plan_dump(spec, rank, n, 1 << 16))
        for s, ws in enumerate(w):
            use = np.zeros(n, int)
            for c in range(n - 1):
                for p in peers[c][s][1]:
                    use[p] += 1
            use = np.delete(use, rank)
            assert use.min() == use.max() == ws - 1, (spec, rank, s, use)


def test_link_time_one_seventh_and_priced_near_flat(nv):
    """program_cost: the busiest link of every phase carries 1/7 of single-channel RHD's bytes at N = 8, and
    the model prices rhd:7+pull within 15 % of flat+pull at 256 MiB (single-channel RHD: ~5.8x)."""
    S = 256 << 20
    one = nv.program_cost("rhd+pull", 0, 8, S // 4, links=7)
    seven = nv.program_cost("rhd:7+pull", 0, 8, S // 4, links=7)
    assert seven["link_time_bytes"] == pytest.approx(one["link_time_bytes"] / 7, rel=1e-4)
    assert seven["link_bytes"] == pytest.approx(one["link_bytes"], rel=1e-4)
    assert seven["handoffs"] == one["handoffs"] == 6
    flat = nv.model_cost_us("flat+pull", 8, S)
    assert nv.model_cost_us("rhd:7+pull", 8, S) < 1.15 * flat
    assert nv.model_cost_us("rhd+pull", 8, S) > 4 * flat
    assert nv.model_cost_us("tree:4,2:7+pull", 8, S) < 1.15 * flat


def test_greedy_relabelling_balances_non_power_of_two(nv):
    """N = 6, tree:2,3:5: the greedy relabelling spreads each stage over the links (busiest link per phase
    well below the single-channel tree's)."""
    one = nv.program_cost("tree:2,3+pull", 0, 6, 6 << 20, links=5)
    five = nv.program_cost("tree:2,3:5+pull", 0, 6, 6 << 20, links=5)
    assert five["link_time_bytes"] < 0.5 * one["link_time_bytes"]


def test_parse_and_errors(nv):
    assert "tree:2,2,2:7" in nv.enumerate_plans(8)
    assert "tree:4,2:7" in nv.enumerate_plans(8) and "tree:2,4:7" in nv.enumerate_plans(8)
    assert not any(p.endswith(":7") and p.startswith("tree:8") for p in nv.enumerate_plans(8))
    assert "rank 0 program 'tree:2,2,2:7+pull'" in nv.plan_dump("rhd:7+pull", 0, 8, 4096)
    with pytest.raises(nv.FlexarError):
        nv.simulate("tree:2,2:3", [np.zeros(64, np.int32)] * 5)  # lonely ranks: no channels
    with pytest.raises(nv.FlexarError):
        nv.simulate("rhd:x", [np.zeros(64, np.int32)] * 4)
    for bad in ("tree:4:3+zc", "tree:4:3+bidir"):  # the direct exchanges have no stages to relabel
        with pytest.raises(nv.FlexarError):
            nv.simulate(bad, [np.zeros(64, np.int32)] * 4, grid=6)


def test_message_transport_runs_channelled_trees(nv):
    """+rccl: the channels are flattened in order into grouped send/recv steps, still exact."""
    n = 8
    ins = [np.random.default_rng(r).integers(-99, 99, 10007).astype(np.int32) for r in range(n)]
    want = np.sum(np.stack(ins), 0)
    for o in nv.simulate_msg("rhd:7", ins):
        np.testing.assert_array_equal(o, want)


def test_selector_prices_channelled_trees(nv):
    """Every enumerated channelled tree builds and prices (the selector sees them as candidates)."""
    for n in (4, 6, 8, 12, 16):
        for p in nv.enumerate_plans(n):
            if p.startswith("tree:") and p.count(":") == 2:
                assert nv.model_cost_us(p + "+pull", n, 64 << 20) < 1e20, (n, p)


def test_random_trees_and_channels_exact(nv):
    """Property check over random world sizes, factorizations, channel counts, sizes and all-gather forms: every
    channelled tree the planner accepts sums exactly on every rank (simulator of the device protocol)."""
    from hypothesis import given, settings, strategies as st

    import math

    facts = {n: [p for p in nv.enumerate_plans(n) if p.startswith("tree:") and "," in p and p.count(":") == 1
                 and math.prod(int(w) for w in p[5:].split(",")) == n]  # lonely-rank trees take no channels
             for n in range(4, 17)}
    facts = {n: v for n, v in facts.items() if v}

    @settings(max_examples=60, deadline=None, derandomize=True)
    @given(st.sampled_from(sorted(facts)), st.integers(0, 10 ** 6), st.integers(2, 20), st.integers(1, 6000),
           st.sampled_from(["", "+push", "+pull", "+push+nofuse"]))
    def check(n, pick, C, size, mod):
        base = facts[n][pick % len(facts[n])]
        spec = f"{base}:{C}{mod}"
        ins = [np.random.default_rng(size + r).integers(-99, 99, size).astype(np.int32) for r in range(n)]
        want = np.sum(np.stack(ins), 0)
        stages = base.count(",") + 1
        grid = 2 * min(C, 126 // (2 * stages))  # the planner caps C at the flag-slot budget (2 per stage)
        for r, o in enumerate(nv.simulate(spec, ins, grid=grid, ncalls=2)):
            np.testing.assert_array_equal(o, want, err_msg=f"{spec} n={n} size={size} r={r}")

    check()
