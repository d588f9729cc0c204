"""The OCP MX block-scaled fp8 wire on the GPU ("+mxe4m3" / "+mxe5m2", docs/DESIGN.md §9.2): one launch of
every rank of an in-process group, bit for bit against ops.quant.mx_allreduce_reference (the CPU tests pin
that reference to the host executor), over the lane-interleaved super-groups, the contiguous blocks and the
element-wise tail, the fence and write-through protocols, both parities. The multi-process form is in
test_gpu_multidevice.py (exec kernel, one process per rank).

Reference counterpart: none (the reference moves fp32 only); BASELINE config #5 without its amax pass.
"""
import pytest
import torch

from allreduce_over_mpi_amd.ops.quant import mx_allreduce_reference

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def groups(cuda):
    from allreduce_over_mpi_amd.parallel import LocalGroup

    gs = {n: LocalGroup(n, workspace_bytes=96 << 20) for n in (2, 4, 8)}
    yield gs
    for g in gs.values():
        g.close()


def _xs(n, count, dtype, seed, spread=2.0):
    g = torch.Generator().manual_seed(seed)
    lim = 6e4 if dtype == torch.float16 else 1e30
    return [(torch.randn(count, generator=g) * torch.exp(torch.randn(count, generator=g) * spread)).clamp(-lim, lim)
            .to(dtype) for _ in range(n)]


def _check(grp, xs, spec, op, cuda, reps=2):
    wire = spec.rsplit("+mx", 1)[1]
    want = mx_allreduce_reference(xs, wire, op)
    for _ in range(reps):  # both staging parities
        outs = grp.all_reduce([x.to(cuda) for x in xs], op, algo=spec)
        torch.cuda.synchronize()
        for r, o in enumerate(outs):
            bad = (o.cpu().view(torch.uint8) != want.view(torch.uint8)).nonzero().flatten()
            assert bad.numel() == 0, (spec, op, str(xs[0].dtype), r, bad[:8].tolist(), o.numel())
    grp.check()


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_group_mx_wire_bitwise(cuda, groups, n, dtype):
    # 1000003: interleaved super-groups + contiguous blocks + a 19-element tail per chunk boundary
    for count in (1000003, 4099, 33):
        _check(groups[n], _xs(n, count, dtype, seed=n * 7 + count), "flat+pull+mxe4m3", "avg", cuda)
    _check(groups[n], _xs(n, 65537, dtype, seed=n), "flat+pull+mxe5m2", "sum", cuda)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_group_mx_wire_write_through_and_large(cuda, groups, dtype):
    n = 4
    _check(groups[n], _xs(n, 300001, dtype, seed=5), "flat+pull+wt+mxe4m3", "avg", cuda)
    _check(groups[n], _xs(n, 8 * 1024 * 1024 + 333, dtype, seed=6), "flat+pull+mxe4m3", "avg", cuda, reps=1)


def test_group_mx_wire_keeps_small_blocks(cuda, groups):
    """Blocks 2^-20 .. 2^20 apart: per-block scales keep each block's relative precision, where the
    per-call global scale of "+e4m3" flushes the small blocks (test_mx_wire.py has the CPU form)."""
    n, count = 4, 1 << 20
    g = torch.Generator().manual_seed(9)
    mag = torch.pow(2.0, torch.randint(-20, 21, (count // 32,), generator=g).float()).repeat_interleave(32)
    xs = [torch.randn(count, generator=g) * mag for _ in range(n)]
    exact = torch.stack([x.double() for x in xs]).sum(0)
    mx = groups[n].all_reduce([x.to(cuda) for x in xs], "sum", algo="flat+pull+mxe4m3")[0].cpu().double()
    glob = groups[n].all_reduce_fp8([x.to(cuda) for x in xs], op="sum")[0].cpu().double()
    med = lambda y: float(((y - exact).abs() / exact.abs().clamp_min(1e-30)).median())
    assert med(mx) < 0.05, med(mx)
    assert med(glob) > 10 * med(mx), (med(glob), med(mx))


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_group_mx_reduce_scatter_bitwise(cuda, groups, n, dtype):
    """The MX wire on the flat reduce-scatter, one launch, byte for byte against
    ops.quant.mx_reduce_scatter_reference (block r of every rank: own value first, then the peers)."""
    from allreduce_over_mpi_amd.ops.quant import mx_reduce_scatter_reference

    for m, wire, op in ((250001, "e4m3", "avg"), (4099, "e5m2", "sum")):
        xs = _xs(n, n * m, dtype, seed=n + m)
        want = mx_reduce_scatter_reference(xs, wire, op)
        for _ in range(2):
            outs = [torch.empty(m, device=cuda, dtype=dtype) for _ in range(n)]
            groups[n].collective("reduce_scatter", [x.to(cuda) for x in xs], outs, op=op, algo=f"flat+mx{wire}")
            torch.cuda.synchronize()
            for r, (o, w) in enumerate(zip(outs, want)):
                bad = (o.cpu().view(torch.uint8) != w.view(torch.uint8)).nonzero().flatten()
                assert bad.numel() == 0, (n, m, wire, op, r, bad[:8].tolist())
    groups[n].check()


def test_kernel_info_reports_every_executor_class(cuda):
    """flexar_kernel_info for the untyped, fp32-partials, global-scale fp8 and MX executors: each fits at least
    one 512-thread workgroup per CU (the protocol's co-residency assumption, choose_grid)."""
    from allreduce_over_mpi_amd import _native as nv

    for dt, kind in (("float32", 0), ("bfloat16", 3), ("float32", 4), ("float32", 6), ("bfloat16", 7)):
        for proto in (0, 2):
            k = nv.kernel_info(dt, "sum", kind, proto)
            assert k["blocks_per_cu"] >= 1 and 0 < k["vgprs"] <= 256, (dt, kind, proto, k)


def test_production_executors_scratch_free_one_workgroup_per_cu(cuda):
    """Round 6 (profiles/r6_mx_nd/): every production executor runs without scratch, and at one 512-thread workgroup
    per CU. Covered: the untyped executor in every protocol, LL, fp32 partials, the global-scale fp8 wire and the
    fan-in-8 MX wire. Scratch had come from two sources: the fan-in-8 MX spills, and copying the by-value context.
    A kernel at <= 128 VGPRs would pack two workgroups per CU."""
    from allreduce_over_mpi_amd import _native as nv

    cases = [(dt, 0, p) for dt in ("float32", "bfloat16") for p in (0, 1, 2)]
    cases += [(dt, 1, 0) for dt in ("float32", "bfloat16")]
    cases += [("bfloat16", 3, p) for p in (0, 2)]
    cases += [(dt, k, p) for dt in ("float32", "bfloat16") for k in (4, 5, 6, 7) for p in (0, 2)]
    for dt, kind, proto in cases:
        k = nv.kernel_info(dt, "sum", kind, proto)
        assert k["scratch_bytes"] == 0, (dt, kind, proto, k)
        if kind != 1:
            assert k["blocks_per_cu"] == 1, (dt, kind, proto, k)


def test_default_spec_wire_applies_only_where_it_can(cuda, monkeypatch):
    """FLEXAR_ALGO=flat+mxe4m3 as the communicator default: float SUM / AVG allreduces and reduce-scatters take
    the MX wire; integer / MAX allreduces and the all-gather run untyped instead of failing."""
    from allreduce_over_mpi_amd.parallel import LocalGroup

    monkeypatch.setenv("FLEXAR_ALGO", "flat+mxe4m3")
    n, count = 4, 4096
    grp = LocalGroup(n, workspace_bytes=32 << 20)
    try:
        xs = _xs(n, count, torch.float32, seed=3)
        outs = grp.all_reduce([x.to(cuda) for x in xs], "avg")
        want = mx_allreduce_reference(xs, "e4m3", "avg")
        assert torch.equal(outs[0].cpu().view(torch.uint8), want.view(torch.uint8))
        ints = [torch.full((count,), r + 1, dtype=torch.int32, device=cuda) for r in range(n)]
        assert bool((grp.all_reduce(ints, "sum")[0] == n * (n + 1) // 2).all())
        fl = [torch.full((count,), float(r), device=cuda) for r in range(n)]
        assert bool((grp.all_reduce(fl, "max")[0] == n - 1).all())
        ag_in = [torch.full((count,), float(r), device=cuda) for r in range(n)]
        ag_out = [torch.empty(n * count, device=cuda) for _ in range(n)]
        grp.collective("all_gather", ag_in, ag_out)
        assert torch.equal(ag_out[1].cpu(), torch.arange(n).float().repeat_interleave(count))
        grp.check()
    finally:
        grp.close()


@pytest.mark.parametrize("wire", ["e4m3", "e5m2"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mx_codec_matches_reference(cuda, wire, dtype):
    """Native MX message codec (csrc/src/k_mx_codec.hip, the hierarchical cross-node step): pack is bitwise
    [mx_quantize bytes | scale bytes]; unpack_sum is bitwise the dequantised rows summed in order. Sizes off
    the 32-element block and an all-zero block included."""
    from allreduce_over_mpi_amd.ops.quant import (mx_dequantize, mx_message_bytes, mx_pack, mx_quantize,
                                                  mx_unpack_sum)

    for n in (1, 31, 33, 4096, 100003):
        xs = []
        for k in range(3):
            x = torch.randn(n, generator=torch.Generator().manual_seed(n + k)) * 10.0 ** (k - 1)
            x[: min(n, 32)] = 0.0 if k == 1 else x[: min(n, 32)]
            xs.append(x.to(dtype))
        msgs = torch.stack([mx_pack(x.cuda(), wire) for x in xs])
        assert msgs.shape == (3, mx_message_bytes(n))
        want_sum = None
        for k, x in enumerate(xs):
            q, sb = mx_quantize(x.float(), wire)
            want = torch.cat([q.view(torch.uint8), sb.to(torch.uint8)])
            assert torch.equal(msgs[k].cpu(), want), (n, k)
            v = mx_dequantize(q, sb, n)
            want_sum = v if want_sum is None else want_sum + v
        got = mx_unpack_sum(msgs, n, wire).cpu()
        assert torch.equal(got, want_sum), (n, int((got != want_sum).sum()))
        # AVG's 1 / world fused into the same pass (hierarchical.py): bitwise the fp32 multiply after the sum
        got = mx_unpack_sum(msgs, n, wire, post=1.0 / 3).cpu()
        assert torch.equal(got, want_sum * (1.0 / 3)), (n, int((got != want_sum * (1.0 / 3)).sum()))
        # unaligned message rows (the all-gathered rows are mx_message_bytes(n) apart): the 16-B accesses
        mb = mx_message_bytes(n)
        buf = torch.zeros(3 * mb + 8, dtype=torch.uint8, device=cuda)
        buf[3:3 + 3 * mb] = msgs.reshape(-1)
        got = mx_unpack_sum(buf[3:3 + 3 * mb].view(3, mb), n, wire).cpu()  # base 3 B past an allocation
        assert torch.equal(got, want_sum), n


@pytest.mark.parametrize("wire", ["e4m3", "e5m2"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_mx_codec_non_finite_matches_reference(cuda, wire, dtype):
    """the pack's scaled converts (v_cvt_scalef32_pk_*) against ops.quant.mx_quantize on blocks holding
    +Inf, -Inf and NaN - whole blocks and the partial tail block - byte for byte (values and scale bytes), and
    unpack_sum against mx_dequantize of the same bytes (NaN positions compared as NaN)."""
    from allreduce_over_mpi_amd.ops.quant import mx_dequantize, mx_pack, mx_quantize, mx_unpack_sum

    for n in (96, 100, 4096 + 17):
        x = torch.randn(n, generator=torch.Generator().manual_seed(n)) * 3.0
        x[5] = float("inf")              # block 0: +Inf among finite values
        x[40] = float("-inf")            # block 1: -Inf
        x[70] = float("nan")             # block 2: NaN
        x[n - 2] = float("nan")          # the tail block (n = 100, 4113) or the last whole one
        x[n - 1] = float("inf")
        x = x.to(dtype)
        msg = mx_pack(x.cuda(), wire).cpu()
        q, sb = mx_quantize(x.float(), wire)
        want = torch.cat([q.view(torch.uint8), sb.to(torch.uint8)])
        diff = (msg != want).nonzero().flatten().tolist()
        assert not diff, (n, [(i, int(msg[i]), int(want[i])) for i in diff[:8]])
        got = mx_unpack_sum(msg.cuda().unsqueeze(0), n, wire).cpu()
        ref = mx_dequantize(q, sb, n)
        assert torch.equal(torch.isnan(got), torch.isnan(ref)), n
        fin = ~torch.isnan(ref)
        assert torch.equal(got[fin], ref[fin]), n
