"""OCP MX block-scaled fp8 wire ("+mxe4m3" / "+mxe5m2", docs/DESIGN.md §9.2) on the CPU: the host executor
(host_exec.hpp host_xfer_mxb, the device executor's semantics element for element) against an independent
torch reference (ops/quant.py mx_allreduce_reference), bit for bit; the planner's scale shadow; and the
accuracy gain over the per-call global scale on data whose magnitude varies block to block.

Reference counterpart: none - the reference moves fp32 only (allreduce_over_mpi/mpi_mod.hpp reduce_sum);
this is BASELINE config #5's compressed wire without its amax pass.
"""
import numpy as np
import pytest
import torch

from allreduce_over_mpi_amd import _native as nv
from allreduce_over_mpi_amd.ops.quant import (fp8_wire_scale, mx_allreduce_reference, mx_quantize, mx_round,
                                              mx_scale_bytes)

DT = {torch.float32: "float32", torch.bfloat16: "bfloat16", torch.float16: "float16"}


def _raw(x):
    return x.numpy() if x.dtype == torch.float32 else x.view(torch.int16).numpy().view(np.uint16)


def _inputs(n, count, dt, seed, spread=3.0):
    g = torch.Generator().manual_seed(seed)
    lim = 6e4 if dt == torch.float16 else 1e30
    return [(torch.randn(count, generator=g) * torch.exp(torch.randn(count, generator=g) * spread)).clamp(-lim, lim).to(dt)
            for _ in range(n)]


def test_scale_byte_rule():
    x = torch.tensor([448.0] + [0.0] * 31 + [449.0] + [0.0] * 31 + [1.0] + [0.0] * 31 + [0.0] * 32)
    sb = mx_scale_bytes(x, "e4m3").tolist()
    assert sb == [127, 128, 119, 1]  # 448 fits at 2^0, 449 needs 2^1, 1.0 -> 2^-8 (1 * 256 <= 448), zeros clamp
    assert mx_scale_bytes(torch.tensor([57344.0] + [0.0] * 31), "e5m2").tolist() == [127]
    q, _ = mx_quantize(torch.tensor([449.0, -300.0] + [0.0] * 30), "e4m3")
    assert q.float()[:2].tolist() == [224.0, -144.0]  # / 2^1; -150 rounds to -144 (step 16 in [128, 256))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_host_executor_matches_reference_bitwise(dt, n):
    for count in (33, 1000, 32 * 7 + 5, 4096):
        xs = _inputs(n, count, dt, seed=count + n)
        for wire in ("e4m3", "e5m2"):
            for op in ("sum", "avg"):
                outs = nv.simulate_mx(f"flat+pull+mx{wire}", [_raw(x) for x in xs], DT[dt], op=op, grid=3)
                want = _raw(mx_allreduce_reference(xs, wire, op))
                for r, o in enumerate(outs):
                    bad = np.nonzero(o.view(np.uint8) != want.view(np.uint8))[0]
                    assert bad.size == 0, (n, count, DT[dt], wire, op, r, bad[:8])


def test_program_has_a_scale_shadow_and_only_flat_schedules():
    dump = nv.plan_dump("flat+pull+mxe4m3", 1, 4, 4096)
    assert "wire type mx e4m3" in dump and "block scales at" in dump
    shadow = int(dump.split("block scales at ")[1].split()[0].rstrip(","))
    stg = int(dump.split("staging ")[1].split()[0])
    assert shadow >= 8192 and stg >= shadow + 8192 // 32  # one byte per 32 payload bytes, after the payload
    for bad in ("ring+mxe4m3", "rhd+mxe4m3"):
        with pytest.raises(nv.FlexarError):
            nv.simulate_mx(bad, [np.ones(256, np.float32)] * 4, "float32")


def test_block_scales_beat_one_global_scale_on_varied_magnitudes():
    """Blocks 2^-20 .. 2^20 apart: one per-call scale (fp8_max / (N * amax)) flushes the small blocks to zero
    or subnormals; per-block scales keep every block at fp8's relative precision."""
    n, count = 4, 4096
    g = torch.Generator().manual_seed(7)
    mag = torch.pow(2.0, torch.randint(-20, 21, (count // 32,), generator=g).float()).repeat_interleave(32)
    xs = [torch.randn(count, generator=g) * mag for _ in range(n)]
    exact = torch.stack([x.double() for x in xs]).sum(0)
    mx = torch.from_numpy(nv.simulate_mx("flat+pull+mxe4m3", [x.numpy() for x in xs], "float32")[0]).double()
    amax = max(float(x.abs().max()) for x in xs)
    glob = torch.from_numpy(nv.simulate_mx("flat+pull+e4m3", [x.numpy() for x in xs], "float32",
                                           pre=fp8_wire_scale(n, amax))[0]).double()
    rel = lambda y: float(((y - exact).abs() / exact.abs().clamp_min(1e-30)).median())
    assert rel(mx) < 0.05  # e4m3: 3 mantissa bits, a few roundings
    assert rel(glob) > 10 * rel(mx)


def test_mx_round_is_idempotent():
    x = _inputs(1, 999, torch.float32, seed=3)[0]
    y = mx_round(x, "e4m3")
    assert torch.equal(mx_round(y, "e4m3"), y)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_reduce_scatter_mx_matches_reference_bitwise(n):
    """The MX wire on the flat reduce-scatter (FSDP / ZeRO gradient shards): quantising pushes, the owner
    sums its own value first and then the peers' in rank order, no second rounding of its block."""
    from allreduce_over_mpi_amd.ops.quant import mx_reduce_scatter_reference

    for dt in (torch.float32, torch.bfloat16):
        for m in (33, 4099):
            xs = _inputs(n, n * m, dt, seed=m + n)
            for wire, op in (("e4m3", "avg"), ("e5m2", "sum")):
                outs = nv.simulate_coll("reduce_scatter", f"flat+mx{wire}", [_raw(x) for x in xs], m, dtype=DT[dt],
                                        op=op, grid=3)
                for r, (o, w) in enumerate(zip(outs, mx_reduce_scatter_reference(xs, wire, op))):
                    assert np.array_equal(o.view(np.uint8), _raw(w).view(np.uint8)), (n, m, DT[dt], wire, op, r)


def test_mx_wire_only_on_allreduce_and_reduce_scatter():
    ins = [np.ones(4 * 256, np.float32)] * 4
    for coll in ("all_gather", "all_to_all"):
        with pytest.raises(nv.FlexarError):
            nv.simulate_coll(coll, "flat+mxe4m3", [np.ones(256 if coll == "all_gather" else 1024, np.float32)] * 4,
                             256)
    with pytest.raises(nv.FlexarError):  # the ring reduce-scatter has no typed form
        nv.simulate_coll("reduce_scatter", "ring+mxe4m3", ins, 256)
