"""Every algorithm / topology / geometry executed by the CPU simulator of the
device protocol (the exact op programs the gfx950 kernel runs, one thread per
(rank, workgroup), real flags/epochs/parity) against a numpy reference.

Mirrors the survey's black-box verification of the reference:
sizes {1,5,35,1000,1001,65539}, in/out of place, N = 2..8 on every topology,
primes, N = 21 (where the reference's flat fan-in > 20 produced garbage, D3).
"""
import numpy as np
import pytest

SIZES = [1, 5, 35, 1000, 1001, 65539]


def topologies(n):
    from allreduce_over_mpi_amd import _native as nv

    out = ["flat", "flat+push", "ring", "oneshot", "flat+nofuse"]
    out += [p for p in nv.enumerate_plans(n) if p.startswith("tree:") or p.startswith("ring:")]
    out += [p + "+push" for p in nv.enumerate_plans(n) if p.startswith("tree:") and "," in p]
    return sorted(set(out))


def channels_of(spec):
    """C of "ring:C" / "tree:a,b:C" / "rhd:C" (1 otherwise)."""
    head = spec.split("+")[0]
    if head.startswith("ring:") or head.startswith("rhd:"):
        return int(head.split(":")[1])
    return int(head.split(":")[2]) if head.startswith("tree:") and head.count(":") == 2 else 1


def ref_sum(ins):
    return np.sum(np.stack(ins).astype(np.float64), 0)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_all_topologies_f32(nv, n):
    rng = np.random.default_rng(n)
    for spec in topologies(n):
        chans = channels_of(spec)
        for size in SIZES:
            ins = [rng.standard_normal(size).astype(np.float32) for _ in range(n)]
            for in_place in (False, True):
                outs = nv.simulate(spec, ins, grid=max(2, chans) if chans == 1 else chans * 2, ncalls=3,
                                   in_place=in_place)
                ref = ref_sum(ins)
                for r, o in enumerate(outs):
                    np.testing.assert_allclose(o, ref, rtol=1e-5, atol=1e-4, err_msg=f"{spec} n={n} size={size} r={r}")


@pytest.mark.parametrize("n,spec", [(21, "flat"), (21, "tree:3,7"), (21, "ring"), (16, "tree:2,2,2,2"),
                                    (16, "tree:4,4+push"), (12, "tree:2,3,2"), (9, "tree:3,3"),
                                    (12, "oneshot"), (16, "oneshot"), (16, "flat+push"), (11, "flat+push")])
def test_wide_and_prime(nv, n, spec):
    rng = np.random.default_rng(7)
    ins = [rng.integers(-1000, 1000, 4099).astype(np.int64) for _ in range(n)]
    outs = nv.simulate(spec, ins, grid=2, ncalls=2)
    ref = np.sum(np.stack(ins), 0)
    for o in outs:
        np.testing.assert_array_equal(o, ref)


@pytest.mark.parametrize("op", ["sum", "prod", "max", "min", "band", "bor", "bxor"])
@pytest.mark.parametrize("dt", ["int32", "uint8", "int64", "int16"])
def test_integer_ops(nv, op, dt):
    rng = np.random.default_rng(1)
    n = 4
    ins = [rng.integers(0, 100, 777).astype(dt) for _ in range(n)]
    fn = {"sum": np.add, "prod": np.multiply, "max": np.maximum, "min": np.minimum, "band": np.bitwise_and,
          "bor": np.bitwise_or, "bxor": np.bitwise_xor}[op]
    ref = ins[0].copy()
    for x in ins[1:]:
        ref = fn(ref, x).astype(dt)
    for spec in ("flat", "ring", "rhd", "oneshot"):
        outs = nv.simulate(spec, ins, op=op, grid=3, ncalls=2)
        for o in outs:
            np.testing.assert_array_equal(o, ref, err_msg=f"{spec} {op} {dt}")


def test_float_ops_and_avg(nv):
    rng = np.random.default_rng(2)
    n = 8
    ins = [rng.standard_normal(3001).astype(np.float64) for _ in range(n)]
    st = np.stack(ins)
    for op, ref in (("max", st.max(0)), ("min", st.min(0)), ("avg", st.mean(0)), ("sum", st.sum(0))):
        for spec in ("flat", "ring:4", "tree:2,4", "oneshot"):
            outs = nv.simulate(spec, ins, op=op, grid=4, ncalls=2)
            for o in outs:
                np.testing.assert_allclose(o, ref, rtol=1e-12, atol=1e-12, err_msg=f"{spec} {op}")
    outs = nv.simulate("flat", ins, op="sum", grid=2, scale=0.5)
    np.testing.assert_allclose(outs[0], st.sum(0) * 0.5, rtol=1e-12)


def test_unsupported_combinations(nv):
    ins = [np.ones(8, np.float32)] * 2
    with pytest.raises(nv.FlexarError):
        nv.simulate("flat", ins, op="band")   # bitwise on floats (reference: exit(1))
    ins = [np.ones(8, np.int32)] * 2
    with pytest.raises(nv.FlexarError):
        nv.simulate("flat", ins, op="avg")


def _bf16_bits(x):
    import torch

    return torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)


def _from_bf16_bits(b):
    import torch

    return torch.from_numpy(b.view(np.int16)).view(torch.bfloat16).float().numpy()


def test_bf16_fp32_accumulation(nv):
    rng = np.random.default_rng(3)
    n = 8
    xs = [rng.standard_normal(5000).astype(np.float32) for _ in range(n)]
    bits = [_bf16_bits(x) for x in xs]
    exact = np.sum(np.stack([_from_bf16_bits(b) for b in bits]).astype(np.float64), 0)
    for spec in ("flat", "oneshot"):  # single reduction stage: exactly one rounding
        outs = nv.simulate_typed(spec, bits, "bfloat16", grid=2)
        got = _from_bf16_bits(outs[0])
        import torch

        want = torch.from_numpy(exact.astype(np.float32)).to(torch.bfloat16).float().numpy()
        np.testing.assert_array_equal(got, want)


def test_bytes_moved_is_bandwidth_optimal(nv):
    """Remote bytes per rank = 2 (N-1)/N * S for ring/tree (the key structural fact)."""
    import re

    n, count = 8, 1 << 20
    for spec in ("flat+push", "flat+pull", "ring", "ring:4", "rhd+push", "tree:2,4+push", "tree:4,2+pull"):
        dump = nv.plan_dump(spec, 3, n, count)
        moved = 0
        for line in dump.splitlines():
            m = re.match(r"\s+XFER len=(\d+).*\[(.*)\] -> \[(.*)\]", line)
            if not m:
                continue
            ln = int(m.group(1))
            srcs, dsts = m.group(2), m.group(3)
            moved += ln * sum(1 for d in dsts.split(", ") if "@3:" not in d)      # remote writes
            moved += ln * sum(1 for s in srcs.split(" + ") if "@3:" not in s)     # remote reads
        assert moved == 2 * (n - 1) * count // n, (spec, moved)


@pytest.mark.parametrize("n,spec", [(7, "tree:2,3"), (7, "tree:3,2+push"), (5, "tree:2,2"), (7, "tree:6"),
                                    (3, "tree:2"), (13, "tree:2,2,3"), (11, "tree:2,3+push+nofuse")])
def test_lonely_ranks(nv, n, spec):
    """Non-factorable N: trees over P >= N/2 ranks with N - P lonely ranks folded into partners
    (the reference's lonely-node design, dead code there: mpi_mod.hpp:983-1099)."""
    rng = np.random.default_rng(n)
    for size in (1, 35, 1001, 65539):
        ins = [rng.standard_normal(size).astype(np.float32) for _ in range(n)]
        for in_place in (False, True):
            outs = nv.simulate(spec, ins, grid=3, ncalls=3, in_place=in_place)
            ref = ref_sum(ins)
            for o in outs:
                np.testing.assert_allclose(o, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("n", [2, 3, 4, 7, 8])
@pytest.mark.parametrize("spec", ["flat", "ring"])
def test_reduce_scatter_all_gather(nv, n, spec):
    rng = np.random.default_rng(n)
    for m in (1, 5, 1000, 4099):
        ins = [rng.integers(-100, 100, n * m).astype(np.int32) for _ in range(n)]
        outs = nv.simulate_coll("reduce_scatter", spec, ins, m, dtype="int32", grid=3)
        total = np.sum(np.stack(ins), 0)
        for r, o in enumerate(outs):
            np.testing.assert_array_equal(o, total[r * m:(r + 1) * m], err_msg=f"rs {spec} n={n} m={m} r={r}")
        ins = [rng.standard_normal(m).astype(np.float32) for _ in range(n)]
        outs = nv.simulate_coll("all_gather", spec, ins, m, grid=3)
        for o in outs:
            np.testing.assert_array_equal(o, np.concatenate(ins), err_msg=f"ag {spec} n={n} m={m}")


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("spec", ["oneshot", "flat", "flat+wt"])
def test_broadcast(nv, n, spec):
    """Direct multicast and scatter + all-gather from every root, tails included, consecutive calls."""
    rng = np.random.default_rng(n)
    for size in (1, 5, 1001, 65539):
        data = rng.standard_normal(size).astype(np.float32)
        for root in range(n):
            outs = nv.simulate_bcast(spec, data, n, root=root, grid=3, ncalls=3)
            for r, o in enumerate(outs):
                np.testing.assert_array_equal(o, data, err_msg=f"{spec} n={n} size={size} root={root} r={r}")


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_all_to_all(nv, n):
    """Equal-split all-to-all: block p of rank r's input lands in block r of rank p's output."""
    rng = np.random.default_rng(n)
    for m in (1, 7, 1001, 4099):
        ins = [rng.integers(-1000, 1000, n * m).astype(np.int32) for _ in range(n)]
        outs = nv.simulate_coll("all_to_all", "flat", ins, m, dtype="int32", grid=3, ncalls=3)
        for p in range(n):
            want = np.concatenate([ins[r][p * m:(p + 1) * m] for r in range(n)])
            np.testing.assert_array_equal(outs[p], want, err_msg=f"n={n} m={m} p={p}")


@pytest.mark.parametrize("n", [2, 3, 4, 7, 8, 12, 16])
@pytest.mark.parametrize("spec", ["flat+bidir", "flat+bidir+wt", "flat+bidir+nts"])
def test_flat_bidir(nv, n, spec):
    """Direction-balanced flat over staging (planner.hpp build_flat_bidir): the reduce-scatter pulls the
    peers' published IN copies while the same XFER pushes the reduced block into every peer's landing slot.
    Exact sums with uneven tails, out of place and in place, over consecutive calls (both staging parities)."""
    for count in (1, 35, 4099, 10007):
        ins = [np.random.default_rng(7 * r + count).integers(-99, 99, count).astype(np.int32) for r in range(n)]
        want = np.sum(ins, axis=0)
        for in_place in (False, True):
            for o in nv.simulate(spec, ins, ncalls=3, grid=3, in_place=in_place):
                np.testing.assert_array_equal(o, want)


def test_flat_bidir_shape_and_bits(nv):
    d = nv.plan_dump("flat+bidir", 1, 4, 4096, "float32")
    assert "2 flag slots" in d and d.count("XFER") == 7, d  # 3 local copies, 1 pull-reduce-push, 3 copy-outs
    # one XFER reads every peer's staging AND writes every peer's staging: both link directions at once
    fused = [ln for ln in d.splitlines() if "OUT@1" in ln and "STG@0" in ln.split("->")[0]]
    assert len(fused) == 1 and all(f"STG@{p}" in fused[0].split("->")[1] for p in (0, 2, 3)), d
    # rank-order sum: the same bits as the zero-copy forms
    ins = [np.random.default_rng(r).standard_normal(9001).astype(np.float32) * (r + 1) for r in range(8)]
    ref = nv.simulate("flat+zc", ins, grid=2, op="avg")[0]
    for o in nv.simulate("flat+bidir", ins, grid=2, op="avg"):
        assert np.array_equal(o, ref)
    # the message transport has no peer reads: "+bidir" falls back to the push flat's messages there
    assert nv.msg_plan("flat+bidir", 0, 4, 1 << 20, "float32")["messages"] == 6
    with pytest.raises(nv.FlexarError):
        nv.simulate("ring+bidir", [np.zeros(64, np.int32)] * 4)
