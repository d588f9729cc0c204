"""gfx950 kernels on a real MI355X: the standalone reduction kernel and the
complete multi-rank allreduce protocol (LocalGroup: N ranks in one launch on
one GPU — flags, epochs, parity staging, every algorithm) against plain
PyTorch fp32/fp64 references of the same op.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _seq_ref(srcs, op="sum", scale=1.0):
    """Sequential fp32 reduction in source order (the kernel's order), then one rounding."""
    acc = srcs[0].float()
    for s in srcs[1:]:
        f = s.float()
        acc = {"sum": acc + f, "max": torch.maximum(acc, f), "min": torch.minimum(acc, f), "prod": acc * f}[op]
    return acc * scale if scale != 1.0 else acc


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("nsrc", [1, 2, 3, 5, 8, 12])
@pytest.mark.parametrize("n", [1, 37, 4099, 1 << 20])
def test_reduce_kernel_float(cuda, dtype, nsrc, n):
    from allreduce_over_mpi_amd.ops import reduce

    g = torch.Generator(device=cuda).manual_seed(nsrc * 1000 + n)
    srcs = [torch.randn(n, device=cuda, generator=g).to(dtype) for _ in range(nsrc)]
    out = reduce(srcs, "sum")
    torch.cuda.synchronize()
    want = _seq_ref(srcs)
    if dtype in (torch.float32, torch.float64) or nsrc <= 8:
        # single pass: fp32 (fp64) accumulate in source order, one rounding
        torch.testing.assert_close(out.double(), want.to(dtype).double(), rtol=0, atol=0) if dtype != torch.float64 \
            else torch.testing.assert_close(out, sum(s for s in srcs[1:]) + srcs[0], rtol=1e-12, atol=1e-12)
    else:
        torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float8_e4m3fn, torch.float8_e5m2])
def test_reduce_kernel_fp8_scaled(cuda, dtype):
    """fp8 (OCP, gfx950-native) with fused post-scale: fp32 accumulate, one saturating RNE rounding."""
    from allreduce_over_mpi_amd.ops import reduce

    g = torch.Generator(device=cuda).manual_seed(5)
    srcs = [(torch.randn(1 << 16, device=cuda, generator=g) * 4).to(dtype) for _ in range(8)]
    out = reduce(srcs, "sum", scale=0.125)
    torch.cuda.synchronize()
    want = (_seq_ref(srcs) * 0.125).to(dtype)
    assert torch.equal(out.view(torch.uint8), want.view(torch.uint8))


@pytest.mark.parametrize("dtype", [torch.float8_e4m3fn, torch.float8_e5m2])
@pytest.mark.parametrize("nsrc", [2, 3, 8])
def test_reduce_kernel_fp8_saturation_and_nan(cuda, dtype, nsrc):
    """The packed fp8 store (device_exec.hpp fp8_store4) keeps the element store's semantics on every 16-B group
    and on the scalar tail: sums beyond the largest finite saturate to it, infinities too (e5m2), and a NaN
    anywhere in a column gives 0x7f. Finite results are the fp32 source-order sum rounded once (RNE)."""
    from allreduce_over_mpi_amd.ops import reduce

    big = 448.0 if dtype == torch.float8_e4m3fn else 57344.0
    n = 4096 * 3 + 5  # vector groups plus a 5-element scalar tail
    g = torch.Generator(device=cuda).manual_seed(11)
    base = [torch.randn(n, device=cuda, generator=g) * 4 for _ in range(nsrc)]
    for b in base:
        b[::7] = big * 0.75           # columns 0, 7, 14, ...: every source 3/4 of the max -> saturating sums
        b[3::7] = -big * 0.75
    base[0][5::97] = float("nan")
    base[-1][n - 2] = float("nan")    # in the tail
    if dtype == torch.float8_e5m2:
        base[1][11::101] = float("inf")
        base[0][13::101] = float("-inf")
    srcs = [b.to(dtype) for b in base]
    out = reduce(srcs, "sum")
    torch.cuda.synchronize()
    acc = _seq_ref(srcs)
    nan = torch.isnan(acc)
    want = acc.clamp(-big, big).to(dtype).view(torch.uint8)
    got = out.view(torch.uint8)
    assert torch.equal(got[~nan], want[~nan])
    assert bool((got[nan] == 0x7F).all()), got[nan].unique()
    assert int(nan.sum()) > 0 and int((acc.abs() > big).sum()) > 0


@pytest.mark.parametrize("op", ["sum", "max", "min", "band", "bor", "bxor", "prod"])
def test_reduce_kernel_int(cuda, op):
    from allreduce_over_mpi_amd.ops import reduce

    g = torch.Generator(device=cuda).manual_seed(3)
    srcs = [torch.randint(0, 1000, (10007,), device=cuda, generator=g, dtype=torch.int32) for _ in range(4)]
    out = reduce(srcs, op)
    acc = srcs[0].clone()
    for s in srcs[1:]:
        acc = {"sum": acc + s, "max": torch.maximum(acc, s), "min": torch.minimum(acc, s), "band": acc & s,
               "bor": acc | s, "bxor": acc ^ s, "prod": acc * s}[op]
    assert torch.equal(out, acc)


def _specs(n):
    from allreduce_over_mpi_amd import _native as nv

    base = ["flat", "flat+push", "ring", "oneshot", "ll", "flat+nts", "ring:2+nts"]
    base += ["flat+wt", "flat+push+wt", "ring+wt", "ring:2+wt", "oneshot+wt", "dma", "flat+zc", "flat+zc+wt", "flat+zc+push",
             "flat+zc+put", "flat+bidir", "flat+bidir+wt"]
    base += [p for p in nv.enumerate_plans(n) if p.startswith("tree:") or p.startswith("ring:")]
    base += [p + "+push" for p in nv.enumerate_plans(n) if p.startswith("tree:") and "," in p]
    return sorted(set(base))


@pytest.fixture(scope="module")
def groups(cuda):
    """Groups with FLEXAR_PARTIALS=fp32: the tests below assert single rounding of multi-hop schedules (the
    default "auto" policy may round per hop; test_group_partials_auto_default covers it)."""
    import os

    from allreduce_over_mpi_amd.parallel import LocalGroup

    old = os.environ.get("FLEXAR_PARTIALS")
    os.environ["FLEXAR_PARTIALS"] = "fp32"
    try:
        gs = {n: LocalGroup(n, workspace_bytes=64 << 20) for n in (2, 3, 4, 8)}
    finally:
        if old is None:
            os.environ.pop("FLEXAR_PARTIALS")
        else:
            os.environ["FLEXAR_PARTIALS"] = old
    yield gs
    for g in gs.values():
        g.close()


def test_group_partials_auto_default(cuda):
    """The default partials policy ("auto", round 4): a large bf16 RHD at N = 8 may run the per-hop-rounded
    form (three roundings, 1.19x fewer HBM bytes than fp32 partials), a ring keeps fp32 partials (seven
    roundings would be too many). Each rounding errs by at most u = 2^-8 of its partial sum, so the error is
    bounded by (roundings) * u * sum|x| - not by ulps of the final value, which cancellation can make tiny -
    and every rank's result is identical."""
    import os

    from allreduce_over_mpi_amd.parallel import LocalGroup

    assert "FLEXAR_PARTIALS" not in os.environ
    n, count = 8, 8 << 20
    grp = LocalGroup(n, workspace_bytes=256 << 20)
    try:
        g = torch.Generator(device=cuda).manual_seed(5)
        xs = [torch.randn(count, device=cuda, generator=g).to(torch.bfloat16) for _ in range(n)]
        exact = torch.stack([x.double() for x in xs]).sum(0)
        mag = torch.stack([x.double().abs() for x in xs]).sum(0)
        for spec, most in (("rhd", 3), ("ring", 1)):
            outs = grp.all_reduce([x.clone() for x in xs], "sum", algo=spec)
            torch.cuda.synchronize()
            for o in outs:
                assert torch.equal(o.view(torch.int16), outs[0].view(torch.int16)), spec
            # `most` roundings inside the schedule plus the final one
            excess = ((outs[0].double() - exact).abs() - (most + 1) * 2.0 ** -8 * mag).max().item()
            assert excess <= 1e-30, (spec, excess)
        assert _ulps(grp.all_reduce([x.clone() for x in xs], "sum", algo="ring")[0], exact.to(torch.bfloat16)) <= 1
        grp.check()
    finally:
        grp.close()


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_group_allreduce_all_algorithms_f32(cuda, groups, n):
    grp = groups[n]
    for spec in _specs(n):
        for size in (1, 35, 1000, 65539, (1 << 20) + 5):
            g = torch.Generator(device=cuda).manual_seed(size + n)
            xs = [torch.randn(size, device=cuda, generator=g) for _ in range(n)]
            ref = torch.stack([x.double() for x in xs]).sum(0)
            for in_place in (False, True):
                ins = [x.clone() for x in xs]
                outs = None if in_place else [torch.empty_like(x) for x in xs]
                for _ in range(3):  # both staging parities + epoch progression
                    if in_place:
                        for i, x in zip(ins, xs):
                            i.copy_(x)
                    res = grp.all_reduce(ins, "sum", outs=outs, algo=spec)
                    torch.cuda.synchronize()
                    for r, o in enumerate(res):
                        err = (o.double() - ref).abs().max().item()
                        assert err < 1e-4 * math.sqrt(n), f"{spec} n={n} size={size} rank={r} inplace={in_place} err={err}"
    grp.check()


@pytest.mark.parametrize("n,spec", [(4, "rhd:3+pull"), (4, "rhd:3+push"), (8, "rhd:7+pull"), (8, "rhd:7+push"),
                                    (8, "rhd:7+pull+nts"), (8, "rhd:7+pull+wt"), (8, "tree:4,2:7+pull"),
                                    (8, "tree:2,4:7+push+nofuse"), (8, "rhd:3+pull")])
def test_group_channelled_trees_bit_exact(cuda, groups, n, spec):
    """Link-balanced multi-channel trees (planner.hpp build_tree_channels): integer-valued fp32 inputs make every
    partial sum exact, so the device result must EQUAL the fp64 reference - out of place and in place, over
    three consecutive calls (both staging parities), sizes with uneven channel and block tails."""
    grp = groups[n]
    for size in (1, 7, 4099, 65539, (3 << 20) + 17):
        g = torch.Generator(device=cuda).manual_seed(size * 7 + n)
        xs = [torch.randint(-1000, 1000, (size,), device=cuda, generator=g).float() for _ in range(n)]
        ref = torch.stack([x.double() for x in xs]).sum(0)
        for in_place in (False, True):
            ins = [x.clone() for x in xs]
            outs = None if in_place else [torch.empty_like(x) for x in xs]
            for call in range(3):
                if in_place:
                    for i, x in zip(ins, xs):
                        i.copy_(x)
                res = grp.all_reduce(ins, "sum", outs=outs, algo=spec)
                torch.cuda.synchronize()
                for r, o in enumerate(res):
                    assert torch.equal(o.double(), ref), f"{spec} size={size} rank={r} in_place={in_place} call={call}"
    grp.check()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.int32, torch.float64])
def test_group_allreduce_dtypes(cuda, groups, dtype):
    n = 8
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(11)
    if dtype == torch.int32:
        xs = [torch.randint(-1000, 1000, (300007,), device=cuda, generator=g, dtype=dtype) for _ in range(n)]
    else:
        xs = [torch.randn(300007, device=cuda, generator=g).to(dtype) for _ in range(n)]
    ref = torch.stack([x.double() for x in xs]).sum(0)
    for spec in ("flat", "ring:4", "rhd", "tree:2,4+push", "oneshot", "flat+wt", "ring:2+wt", "dma"):
        outs = grp.all_reduce([x.clone() for x in xs], "sum", algo=spec)
        torch.cuda.synchronize()
        for o in outs:
            if dtype == torch.int32:
                assert torch.equal(o.double(), ref)
            elif dtype == torch.float64:
                torch.testing.assert_close(o.double(), ref, rtol=1e-9, atol=1e-9)
            else:
                # every schedule rounds once: multi-hop ones keep fp32 partials by default (typed staging),
                # so the result is within 1 ulp of the correctly rounded exact sum (round 1 needed 8x the
                # dtype's step for ring / RHD / trees)
                assert _ulps(o, ref.to(dtype)) <= 1, (spec, _ulps(o, ref.to(dtype)))


def _ulps(a: torch.Tensor, b: torch.Tensor) -> int:
    """Max distance in units in the last place between two 16/8-bit float tensors of one dtype."""
    bits = {2: torch.int16, 1: torch.int8}[a.element_size()]
    ia, ib = a.view(bits).int(), b.view(bits).int()
    m = (1 << (8 * a.element_size() - 1)) - 1
    oa = torch.where(ia < 0, -(ia & m), ia)
    ob = torch.where(ib < 0, -(ib & m), ib)
    return int((oa - ob).abs().max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float8_e4m3fn])
@pytest.mark.parametrize("spec", ["ring", "ring:4", "ring:7", "rhd", "tree:2,4", "tree:4,2+push", "tree:2,2,2+pull",
                                  "rhd:7+pull", "tree:4,2:7+push"])
def test_group_typed_fp32_partials(cuda, groups, dtype, spec):
    """Multi-hop schedules of 16/8-bit inputs keep partial sums in fp32 staging (exec_mx_kernel with fp32
    wire operands): the device result is within 1 ulp of the exact sum rounded once, i.e. flat's result,
    and identical on every rank. "+rw" restores per-hop rounding (compared for contrast)."""
    n = 8
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(21)
    base = [torch.randn(300007, device=cuda, generator=g) * (2 if dtype == torch.float8_e4m3fn else 1)
            for _ in range(n)]
    xs = [b.to(dtype) for b in base]
    exact = torch.stack([x.double() for x in xs]).sum(0)
    want = exact.float().clamp(-448, 448).to(dtype) if dtype == torch.float8_e4m3fn else exact.to(dtype)
    for _ in range(2):  # both staging parities
        outs = grp.all_reduce([x.clone() for x in xs], "sum", algo=spec)
        torch.cuda.synchronize()
        for o in outs:
            assert torch.equal(o.view(torch.uint8), outs[0].view(torch.uint8)), "ranks disagree"
        assert _ulps(outs[0], want) <= 1, _ulps(outs[0], want)
    flat = grp.all_reduce([x.clone() for x in xs], "sum", algo="flat")[0]
    assert _ulps(outs[0], flat) <= 1
    rw = grp.all_reduce([x.clone() for x in xs], "sum", algo=spec + "+rw")[0]
    torch.cuda.synchronize()
    assert _ulps(rw, want) >= _ulps(outs[0], want)
    grp.check()


def _emulate_fp8_flat(xs, s, op, wire=torch.float8_e4m3fn):
    """torch emulation of the flat+e4m3 program: every contribution quantised with s, fp32 sum with the
    block owner's own first and the peers rotated after it, post-scale, one fp8 rounding, / s."""
    n = len(xs)
    q = [(x.float() * s).to(wire).float() for x in xs]
    count = xs[0].numel()
    split = -(-count // n)
    split = -(-split // 256) * 256
    out = torch.empty(count, device=xs[0].device)
    for k in range(n):
        lo, hi = k * split, min(count, (k + 1) * split)
        if lo >= hi:
            continue
        acc = q[k][lo:hi].clone()
        for jj in range(1, n):
            acc = acc + q[(k + jj) % n][lo:hi]
        if op == "avg":
            acc = acc * (1.0 / n)
        out[lo:hi] = acc.to(wire).float()
    return (out * (1.0 / s)).to(xs[0].dtype)


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("dtype,op", [(torch.float32, "avg"), (torch.bfloat16, "avg"), (torch.float32, "sum"),
                                      (torch.float16, "avg")])
def test_group_fp8_wire_fused_scale(cuda, groups, n, dtype, op):
    """BASELINE config #5 in one launch: fp32/bf16/fp16 buffers, e4m3 on the wire. The executor derives
    s = 448 / (N * global amax) from every rank's amax partials (granule exchange), quantises each
    contribution inside the first transfer and dequantises inside the last. Checked against a torch
    emulation of the same arithmetic (bit-exact up to fp32 association flips) and an fp64 reference."""
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(31 + n)
    xs = [(torch.randn(1000003, device=cuda, generator=g) * (r + 1)).to(dtype) for r in range(n)]
    amax = max(float(x.float().abs().max()) for x in xs)
    from allreduce_over_mpi_amd.ops.quant import fp8_wire_scale

    s = fp8_wire_scale(n, amax)  # the device's pre-scale (device_exec.hpp fp8_scale): the sum never saturates
    want = _emulate_fp8_flat(xs, s, op)
    ref = torch.stack([x.double() for x in xs]).sum(0) / (n if op == "avg" else 1)
    for _ in range(3):  # parities; the amax granules are epoch-tagged
        outs = grp.all_reduce_fp8([x.clone() for x in xs], op=op)
        torch.cuda.synchronize()
        for o in outs:
            assert torch.equal(o, outs[0]), "ranks disagree"
        # s and 1/s are computed in fp32 on the device and in fp64 -> fp32 here: allow that last-bit slack
        mism = (~torch.isclose(outs[0].float(), want.float(), rtol=1e-5, atol=0)).float().mean().item()
        assert mism < 2e-3, mism
        rel = ((outs[0].double() - ref).abs().max() / ref.abs().max()).item()
        assert rel < 0.1, rel  # e4m3: half-ulp 2^-4 of the result + the quantised contributions
    grp.check()


def test_group_flat_bf16_single_rounding(cuda, groups):
    """flat = one reduction stage: every rank gets the fp32-accumulated sum rounded once."""
    n = 8
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(12)
    xs = [torch.randn(65536, device=cuda, generator=g).to(torch.bfloat16) for _ in range(n)]
    outs = grp.all_reduce([x.clone() for x in xs], "sum", algo="flat")
    exact = torch.stack([x.double() for x in xs]).sum(0)
    for o in outs:
        assert (o.double() - exact).abs().max().item() <= (exact.abs() * 2 ** -8).max().item() + 1e-6


def test_group_avg_and_fp8(cuda, groups):
    n = 4
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(13)
    xs = [torch.randn(4096, device=cuda, generator=g) for _ in range(n)]
    outs = grp.all_reduce([x.clone() for x in xs], "avg", algo="flat")
    ref = torch.stack(xs).mean(0)
    for o in outs:
        torch.testing.assert_close(o, ref, rtol=1e-5, atol=1e-6)
    # fp8 e4m3 gradient allreduce with fused 1/N post-scale (BASELINE config #5)
    x8 = [(x * 8).to(torch.float8_e4m3fn) for x in xs]
    exact = (torch.stack([x.float() for x in x8]).sum(0) / n)
    for spec in ("flat", "flat+wt", "dma"):  # one fp32-accumulated reduction stage each
        outs = grp.all_reduce([x.clone() for x in x8], "avg", algo=spec)
        for o in outs:
            assert torch.equal(o.view(torch.uint8), exact.to(torch.float8_e4m3fn).view(torch.uint8)) or \
                (o.float() - exact).abs().max().item() <= 0.0625 * exact.abs().max().item(), spec
    outs = grp.all_reduce([x.clone() for x in xs], "avg", algo="dma")
    for o in outs:
        torch.testing.assert_close(o, ref, rtol=1e-5, atol=1e-6)


def test_group_mixed_engines_sequence(cuda, groups):
    """Executor, LL and copy-engine calls share one staging/epoch protocol: any interleaving (including
    sizes that split into pieces) must stay correct on both parities."""
    n = 4
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(31)
    seq = ["dma", "ll", "flat", "dma", "dma", "ring+wt", "oneshot", "dma", "flat+wt", "ll", "ll", "dma",
           "tree:2,2+push", "dma"]
    for it, spec in enumerate(seq):
        size = [1000, 65539, 300007, (1 << 22) + 3][it % 4]
        xs = [torch.randn(size, device=cuda, generator=g) for _ in range(n)]
        ref = torch.stack([x.double() for x in xs]).sum(0)
        outs = grp.all_reduce([x.clone() for x in xs], algo=spec)
        torch.cuda.synchronize()
        for o in outs:
            assert (o.double() - ref).abs().max().item() < 1e-4, (it, spec, size)
    grp.check()


def test_communicator_single_rank(cuda):
    from allreduce_over_mpi_amd.parallel import Communicator

    c = Communicator(rank=0, world_size=1, workspace_bytes=16 << 20)
    x = torch.randn(12345, device=cuda)
    y = torch.empty_like(x)
    c.all_reduce(x, out=y)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    c.all_reduce(x, op="avg", out=y, scale=2.0)
    torch.cuda.synchronize()
    torch.testing.assert_close(y, 2 * x)
    c.close()


def test_group_varying_grid_between_calls(cuda, groups):
    """Consecutive calls with different grid sizes must agree on one staging parity per call."""
    n = 4
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(21)
    try:
        for it, (grid, size, spec) in enumerate([(8, 300001, "flat"), (32, 1 << 20, "flat"), (4, 5000, "ring"),
                                                 (16, 777777, "rhd"), (8, 300001, "flat+push"), (64, 65536, "ring:2")]):
            grp.set_grid(grid)
            xs = [torch.randn(size, device=cuda, generator=g) for _ in range(n)]
            ref = torch.stack([x.double() for x in xs]).sum(0)
            outs = grp.all_reduce([x.clone() for x in xs], algo=spec)
            torch.cuda.synchronize()
            for o in outs:
                assert (o.double() - ref).abs().max().item() < 1e-4, (it, grid, spec)
        grp.check()
    finally:
        grp.set_grid(0)



@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.int8, torch.float8_e4m3fn,
                                   torch.int32])
@pytest.mark.parametrize("n", [2, 8])
def test_group_ll_protocol(cuda, groups, dtype, n):
    """LL one-shot: 8-B {word, epoch} granules, tails of 1..3 bytes, bit-identical across ranks."""
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(31)
    for size in (1, 3, 1001, 4099, 65537):
        if dtype in (torch.int8, torch.int32):
            xs = [torch.randint(-3, 4, (size,), device=cuda, generator=g, dtype=dtype) for _ in range(n)]
        else:
            xs = [torch.randn(size, device=cuda, generator=g).to(dtype) for _ in range(n)]
        for _ in range(3):
            outs = grp.all_reduce([x.clone() for x in xs], algo="ll")
            torch.cuda.synchronize()
            acc = xs[0].float()
            for x in xs[1:]:
                acc = acc + x.float()
            want = acc.to(dtype)
            for o in outs:
                assert torch.equal(o.view(torch.uint8), outs[0].view(torch.uint8))  # identical on all ranks
                if dtype in (torch.float32, torch.int8, torch.int32):
                    assert torch.equal(o, want), (dtype, size)
                else:
                    assert torch.equal(o.view(torch.uint8), want.view(torch.uint8)), (dtype, size)
    grp.check()


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("spec", ["flat", "ring", "flat+nts", "flat+wt", "ring+wt", "flat+zc", "flat+zc+wt"])
def test_group_reduce_scatter_all_gather(cuda, groups, n, spec):
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(41)
    for m in (1, 37, 100003):
        xs = [torch.randn(n * m, device=cuda, generator=g) for _ in range(n)]
        outs = [torch.empty(m, device=cuda) for _ in range(n)]
        grp.collective("reduce_scatter", xs, outs, algo=spec)
        total = torch.stack([x.double() for x in xs]).sum(0)
        for r, o in enumerate(outs):
            assert (o.double() - total[r * m:(r + 1) * m]).abs().max().item() < 1e-4, (spec, n, m, r)
        ys = [torch.randn(m, device=cuda, generator=g).to(torch.bfloat16) for _ in range(n)]
        gath = [torch.empty(n * m, device=cuda, dtype=torch.bfloat16) for _ in range(n)]
        grp.collective("all_gather", ys, gath, algo=spec)
        cat = torch.cat(ys)
        for o in gath:
            assert torch.equal(o, cat)
    grp.check()


def test_chunk_and_channel_knobs(cuda, monkeypatch):
    """FLEXAR_CHUNK_BYTES splits a call into launches of at most that many bytes; FLEXAR_NCHANNELS sets the
    channel count of a plain ring spec (both read once, at communicator creation)."""
    from allreduce_over_mpi_amd.parallel import LocalGroup

    monkeypatch.setenv("FLEXAR_CHUNK_BYTES", str(1 << 20))
    monkeypatch.setenv("FLEXAR_NCHANNELS", "2")
    monkeypatch.setenv("FLEXAR_ALGO", "ring")
    grp = LocalGroup(4, workspace_bytes=32 << 20)
    try:
        d = grp.describe(1 << 20, torch.float32)
        assert d.startswith("ring:2") and "pieces=4" in d, d
        xs = [torch.randn((1 << 20) + 3, device=cuda) for _ in range(4)]
        ref = torch.stack([x.double() for x in xs]).sum(0)
        for spec in (None, "flat", "ring"):
            outs = grp.all_reduce([x.clone() for x in xs], algo=spec)
            torch.cuda.synchronize()
            for o in outs:
                assert (o.double() - ref).abs().max().item() < 1e-4, spec
        grp.check()
    finally:
        grp.close()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_dma_pipelined_pieces(cuda, monkeypatch, n):
    """Copy-engine allreduce split into many pieces (FLEXAR_CHUNK_BYTES): the pipelined schedule (RS copies
    of piece k+1 while piece k reduces, AG copies of k while k+1 scatters, staging halves reused every
    other piece) gives exact integer-valued sums, in and out of place, over consecutive calls."""
    from allreduce_over_mpi_amd.parallel import LocalGroup

    monkeypatch.setenv("FLEXAR_CHUNK_BYTES", str(256 << 10))
    grp = LocalGroup(n, workspace_bytes=16 << 20)
    try:
        for size in ((1 << 20) + 77, 3 << 20):
            g = torch.Generator(device=cuda).manual_seed(size + n)
            xs = [torch.randint(-50, 50, (size,), device=cuda, generator=g).float() for _ in range(n)]
            ref = torch.stack(xs).sum(0)
            for it in range(3):
                outs = grp.all_reduce([x.clone() for x in xs], algo="dma")
                outs2 = grp.all_reduce([x * 2 for x in xs], outs=[torch.empty_like(x) for x in xs], algo="dma")
                torch.cuda.synchronize()
                for o, o2 in zip(outs, outs2):
                    assert torch.equal(o, ref) and torch.equal(o2, 2 * ref), (size, it)
        grp.check()
    finally:
        grp.close()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_group_broadcast(cuda, groups, n):
    """Broadcast from every root: direct (small/auto) and scatter + all-gather (large/flat), fp32 and bf16,
    with data that changes every call (stale staging would show)."""
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(51)
    for dtype in (torch.float32, torch.bfloat16):
        for size in (3, 4099, 300007):
            for spec in (None, "oneshot", "flat", "flat+wt", "flat+zc"):
                for root in range(n):
                    src = torch.randn(size, device=cuda, generator=g).to(dtype)
                    ins = [src if r == root else torch.zeros_like(src) for r in range(n)]
                    outs = [torch.full_like(src, -1) for _ in range(n)]
                    grp.broadcast(ins, outs, root=root, algo=spec)
                    torch.cuda.synchronize()
                    for r, o in enumerate(outs):
                        assert torch.equal(o, src), (dtype, size, spec, root, r)
    grp.check()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [1, 15, 4096, (1 << 20) + 7])
def test_fp8_compression_kernels(cuda, dtype, n):
    """amax / quantize / dequantize kernels against the PyTorch ops they fuse (bit-exact)."""
    from allreduce_over_mpi_amd.ops import fp8_amax, fp8_dequantize, fp8_quantize

    g = torch.Generator(device=cuda).manual_seed(n)
    x = (torch.randn(n, device=cuda, generator=g) * 3).to(dtype)
    amax = fp8_amax(x)
    torch.cuda.synchronize()
    assert amax.max().item() == x.float().abs().max().item()
    num = 448.0 / 8
    q = fp8_quantize(x, amax, num)
    s = num / amax.max()
    want_q = (x.float() * s).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(q.view(torch.uint8), want_q.view(torch.uint8))
    y = fp8_dequantize(q, amax, num, dtype=dtype)
    want_y = (q.float() * (1.0 / s)).to(dtype)
    assert torch.equal(y, want_y)
    # the round trip is within e4m3's half-step of the largest value
    assert (y.float() - x.float()).abs().max().item() <= amax.max().item() * 2 ** -4 + 1e-6


@pytest.mark.parametrize("n", [2, 4, 8])
def test_group_all_to_all(cuda, groups, n):
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(61)
    for dtype in (torch.float32, torch.bfloat16, torch.int8):
        for m in (1, 37, 100003):
            for it in range(2):  # consecutive calls: both staging halves
                if dtype == torch.int8:
                    ins = [torch.randint(-100, 100, (n * m,), device=cuda, generator=g, dtype=dtype) for _ in range(n)]
                else:
                    ins = [torch.randn(n * m, device=cuda, generator=g).to(dtype) for _ in range(n)]
                for spec in (None, "flat+zc"):  # staging exchange, zero copy into the peers' outputs
                    outs = [torch.empty_like(x) for x in ins]
                    grp.collective("all_to_all", ins, outs, algo=spec)
                    torch.cuda.synchronize()
                    for p in range(n):
                        want = torch.cat([ins[r][p * m:(p + 1) * m] for r in range(n)])
                        assert torch.equal(outs[p], want), (spec, dtype, m, p)
    grp.check()


@pytest.mark.parametrize("dtype,spec", [(torch.bfloat16, "ring"), (torch.bfloat16, "rhd"), (torch.float16, "tree:2,2+push"),
                                        (torch.float8_e4m3fn, "ring")])
def test_group_typed_partials_large_slices(cuda, groups, dtype, spec):
    """Workgroup slices large enough for the typed executor's lane-interleaved super-groups (>= 512 x G
    elements per workgroup, device_exec.hpp xfer_mx) plus their contiguous-group and scalar tails: fp32
    partials still round once (<= 1 ulp of the exact sum) and every rank agrees bit for bit."""
    n = 4
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(5)
    size = 8 * 1024 * 1024 + 4099  # ~2 M elements per ring block: ~32 K per workgroup at grid 64
    xs = [(torch.randn(size, device=cuda, generator=g) * (2 if dtype == torch.float8_e4m3fn else 1)).to(dtype)
          for _ in range(n)]
    exact = torch.stack([x.double() for x in xs]).sum(0)
    want = exact.float().clamp(-448, 448).to(dtype) if dtype == torch.float8_e4m3fn else exact.to(dtype)
    for _ in range(2):
        outs = grp.all_reduce([x.clone() for x in xs], "sum", algo=spec + "+f32")
        torch.cuda.synchronize()
        for o in outs:
            assert torch.equal(o.view(torch.uint8), outs[0].view(torch.uint8)), "ranks disagree"
        assert _ulps(outs[0], want) <= 1, _ulps(outs[0], want)
    grp.check()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_group_fp8_wire_large_slices(cuda, groups, dtype):
    """The fp8 wire's typed transfers over lane-interleaved super-groups (fp32 / bf16 next to e4m3): bit-exact
    against the torch emulation of the same arithmetic, as for the small sizes above."""
    n = 4
    grp = groups[n]
    g = torch.Generator(device=cuda).manual_seed(77)
    xs = [(torch.randn(8 * 1024 * 1024 + 333, device=cuda, generator=g) * (r + 1)).to(dtype) for r in range(n)]
    amax = max(float(x.float().abs().max()) for x in xs)
    from allreduce_over_mpi_amd.ops.quant import fp8_wire_scale

    s = fp8_wire_scale(n, amax)
    want = _emulate_fp8_flat(xs, s, "avg")
    for _ in range(2):
        outs = grp.all_reduce_fp8([x.clone() for x in xs], op="avg")
        torch.cuda.synchronize()
        for o in outs:
            assert torch.equal(o, outs[0]), "ranks disagree"
        mism = (~torch.isclose(outs[0].float(), want.float(), rtol=1e-5, atol=0)).float().mean().item()
        assert mism < 2e-3, mism
    grp.check()


@pytest.mark.parametrize("dtype,offsets", [(torch.float32, ((1, 1), (1, 2), (3, 0), (2, 2))),
                                           (torch.bfloat16, ((1, 1), (1, 3), (0, 5)))])
def test_group_misaligned_views(cuda, groups, dtype, offsets):
    """Tensor views at element offsets (+4 / +8 / +12 B fp32, +2 / +6 / +10 B bf16; input and output
    misaligned alike or differently) take the 16-B vector path with unaligned accesses
    and stay bit-exact against the fp32 torch sum (small integers: every sum is exact in the dtype)."""
    n = 4
    grp = groups[n]
    specs = ["flat", "flat+push", "ring", "ring:3", "rhd", "tree:2,2+pull", "oneshot", "ll", "flat+wt", "dma"]
    if dtype == torch.bfloat16:
        specs += ["ring+f32", "rhd+f32"]
    for size in (1000, 65539, (1 << 20) + 5):
        for oi, oo in offsets:
            bufs = [torch.zeros(size + 16, device=cuda, dtype=dtype) for _ in range(n)]
            obufs = [torch.zeros(size + 16, device=cuda, dtype=dtype) for _ in range(n)]
            base = torch.arange(size, device=cuda, dtype=torch.int32) % 61
            ref = (base * n + n * (n - 1) // 2).to(torch.float32)
            for spec in specs:
                if spec == "ll" and size > 70000:
                    continue
                ins = [b[oi:oi + size] for b in bufs]
                outs = [b[oo:oo + size] for b in obufs]
                for r, x in enumerate(ins):
                    x.copy_((base + r).to(dtype))
                assert (ins[0].data_ptr() % 16 != 0) or (outs[0].data_ptr() % 16 != 0) or oi == oo == 0
                for _ in range(2):  # both staging parities
                    res = grp.all_reduce(ins, "sum", outs=outs, algo=spec)
                    torch.cuda.synchronize()
                    for r, o in enumerate(res):
                        assert torch.equal(o.float(), ref), (spec, size, oi, oo, r,
                                                             (o.float() - ref).abs().max().item())
                # the bytes around the views are untouched
                for b in obufs:
                    assert not b[:oo].any() and not b[oo + size:].any(), (spec, size, oi, oo)
    grp.check()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_group_chunked_work_split_exact(cuda, n):
    """The executor's round-robin chunk split of large spans (set_xfer_chunk / FLEXAR_EXEC_INTERLEAVE,
    device_exec.hpp DevCtx::ichunk): with a small grid every span of these buffers is chunked, a tail chunk is
    partial, and every schedule family - staging, push / pull, rings, trees, write-through, typed partials, the
    fp8 and MX wires - must give exactly what the slice split gives (same arithmetic per element)."""
    from allreduce_over_mpi_amd.parallel import LocalGroup

    grp = LocalGroup(n, workspace_bytes=256 << 20)
    try:
        size = 5 * 8192 * 16 * n + 12345  # spans of > 4 x grid x chunk elements, and a partial last chunk
        g = torch.Generator(device=cuda).manual_seed(17 + n)
        xs = [torch.randn(size, device=cuda, generator=g) for _ in range(n)]
        xb = [x.to(torch.bfloat16) for x in xs]
        specs = ["flat+pull", "flat+push", "ring", "flat+pull+wt", "flat+pull+mxe4m3"] + (["rhd+pull", "tree:2,4+push"]
                                                                                         if n == 8 else [])
        for spec in specs:
            for data in (xs, xb):
                outs = {}
                for chunk in (0, 8192):
                    grp.set_grid(16)
                    grp.set_xfer_chunk(chunk)
                    for _ in range(2):  # both staging parities
                        outs[chunk] = grp.all_reduce([x.clone() for x in data], "sum", algo=spec)
                    torch.cuda.synchronize()
                for r in range(n):
                    assert torch.equal(outs[0][r], outs[8192][r]), (spec, data[0].dtype, r)
        # the global-scale fp8 wire (amax pass + one launch)
        outs = {}
        for chunk in (0, 8192):
            grp.set_xfer_chunk(chunk)
            outs[chunk] = grp.all_reduce_fp8([x.clone() for x in xs], op="avg")
            torch.cuda.synchronize()
        for r in range(n):
            assert torch.equal(outs[0][r], outs[8192][r]), ("fp8", r)
        grp.set_xfer_chunk(0)
        grp.set_grid(0)
        grp.check()
    finally:
        grp.close()
