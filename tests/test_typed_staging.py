"""Typed staging on the CPU simulator (planner.hpp typed operands, host_exec.hpp host_xfer_typed).

* "+f32": multi-hop schedules (ring, RHD, mixed-radix trees) of bf16 / fp8 inputs keep their partial
  sums in fp32 staging, so the result is rounded once - the flat schedule's single rounding - instead of
  once per hop.
* "+e4m3" / "+e5m2": an fp32 / bf16 allreduce with fp8 on the links; the pre-scale s and the post-scale
  1/s are fused into the first and last transfers (BASELINE config #5). Checked bit-exactly against a
  torch emulation of the same quantisation.
The device kernels run the same programs (tests/test_gpu_kernels.py::test_typed_*).
"""
import numpy as np
import pytest
import torch

from allreduce_over_mpi_amd import _native as nv


def _bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16).copy()


def _from_bf16_bits(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16).float()


def _ulps_bf16(a: torch.Tensor, b: torch.Tensor) -> int:
    ia = a.to(torch.bfloat16).view(torch.int16).int()
    ib = b.to(torch.bfloat16).view(torch.int16).int()
    # same sign in these tests (sums of positives + mixed are compared on the ordered integer line)
    oa = torch.where(ia < 0, -(ia & 0x7FFF), ia)
    ob = torch.where(ib < 0, -(ib & 0x7FFF), ib)
    return int((oa - ob).abs().max())


@pytest.mark.parametrize("n,spec", [(8, "ring+f32"), (8, "ring:2+f32"), (8, "rhd+f32"), (8, "tree:2,4+f32"),
                                    (8, "tree:4,2+pull+f32"), (4, "ring+f32"), (6, "tree:3,2+f32"),
                                    (8, "tree:2,2,2+push+f32")])
def test_fp32_partials_round_once(n, spec):
    count = 5003  # uneven tail blocks
    g = torch.Generator().manual_seed(11)
    xs = [torch.randn(count, generator=g) * (1 + r) for r in range(n)]
    ins = [_bf16_bits(x) for x in xs]
    exact = torch.stack([_from_bf16_bits(a).double() for a in ins]).sum(0)
    outs = nv.simulate_mx(spec, ins, "bfloat16", grid=2, ncalls=3)
    flat = nv.simulate_mx("flat", ins, "bfloat16", grid=2, ncalls=3)  # single rounding reference
    for r in range(n):
        got = _from_bf16_bits(outs[r])
        assert torch.equal(got, _from_bf16_bits(outs[0])), "ranks disagree"
        # one rounding of an fp32 sum: at most 1 bf16 ulp from the correctly rounded exact sum, and from flat
        assert _ulps_bf16(got, exact.float()) <= 1
        assert _ulps_bf16(got, _from_bf16_bits(flat[0])) <= 1


def test_round_per_hop_is_worse_than_fp32_partials():
    n, count = 8, 4099
    g = torch.Generator().manual_seed(5)
    ins = [_bf16_bits(torch.randn(count, generator=g)) for _ in range(n)]
    exact = torch.stack([_from_bf16_bits(a).double() for a in ins]).sum(0).float()
    per_hop = _from_bf16_bits(nv.simulate_mx("ring+rw", ins, "bfloat16", grid=2)[0])
    once = _from_bf16_bits(nv.simulate_mx("ring+f32", ins, "bfloat16", grid=2)[0])
    assert _ulps_bf16(once, exact) <= 1
    assert _ulps_bf16(per_hop, exact) > 1  # the per-hop rounding the default now avoids


def test_fp8_inputs_with_fp32_partials():
    n, count = 8, 2051
    g = torch.Generator().manual_seed(2)
    xs = [(torch.randn(count, generator=g) * 4).to(torch.float8_e4m3fn) for _ in range(n)]
    ins = [x.view(torch.uint8).numpy().copy() for x in xs]
    exact = torch.stack([x.double() for x in xs]).sum(0)
    got = nv.simulate_mx("rhd+f32", ins, "fp8_e4m3", grid=2)
    flat = nv.simulate_mx("flat", ins, "fp8_e4m3", grid=2)
    a = torch.from_numpy(got[0]).view(torch.float8_e4m3fn).float()
    b = torch.from_numpy(flat[0]).view(torch.float8_e4m3fn).float()
    want = exact.float().clamp(-448, 448).to(torch.float8_e4m3fn).float()
    assert torch.equal(a, b) or (a - b).abs().max() <= (want.abs() * 0.0625).max()
    # one rounding: the rounded exact sum, except where the fp32 sum itself sits on a rounding boundary
    assert (a != want).float().mean() < 0.01


def _emulate_fp8_flat(xs, s, op, wire=torch.float8_e4m3fn, io=torch.float32):
    """Torch emulation of the flat+e4m3 program: every contribution quantised with s, fp32 sum (owner's own
    block first, then peers in rotated order), scale, one fp8 rounding, dequantised by 1/s."""
    n = len(xs)
    q = [(x.float() * s).to(wire).float() for x in xs]
    count = xs[0].numel()
    split = -(-count // n)
    split = -(-split // 256) * 256  # planner alignment (units of 1 byte for an fp8 wire)
    out = torch.empty(count)
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
    return (out * (1.0 / s)).to(io).float()


@pytest.mark.parametrize("n,op,io", [(8, "sum", "float32"), (4, "avg", "float32"), (8, "avg", "bfloat16"),
                                     (2, "sum", "bfloat16")])
def test_fp8_wire_flat(n, op, io):
    count = 10007
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(count, generator=g) * (r + 1) for r in range(n)]
    tio = getattr(torch, io)
    xs = [x.to(tio) for x in xs]
    amax = max(float(x.float().abs().max()) for x in xs)
    s = 448.0 / (n * amax * 1.0625)  # the device's e4m3 headroom (device_exec.hpp fp8_scale)
    ins = [x.view(torch.int16).numpy().view(np.uint16).copy() if io == "bfloat16" else x.numpy().copy() for x in xs]
    outs = nv.simulate_mx("flat+pull+e4m3", ins, io, op=op, grid=2, ncalls=3, pre=s)
    want = _emulate_fp8_flat(xs, s, op, io=tio)
    for r in range(n):
        got = _from_bf16_bits(outs[r]) if io == "bfloat16" else torch.from_numpy(outs[r]).float()
        if r == 0:
            first = got
        assert torch.equal(got, first), "ranks disagree"
        mism = (~torch.isclose(got, want, rtol=1e-5, atol=0)).float().mean().item()  # 1/s: fp32 here vs fp64
        assert mism < 2e-3, mism  # fp32 sums in another association order can flip an fp8 rounding
        ref = torch.stack([x.double() for x in xs]).sum(0) / (n if op == "avg" else 1)
        assert ((got.double() - ref).abs().max() / ref.abs().max()).item() < 0.1


def test_fp8_wire_rejects_multi_hop_and_wide_groups():
    ins = [np.zeros(64, np.float32) for _ in range(8)]
    for spec in ("ring+e4m3", "rhd+e4m3", "oneshot+e4m3"):
        with pytest.raises(nv.FlexarError):
            nv.simulate_mx(spec, ins, "float32", pre=1.0)
    with pytest.raises(nv.FlexarError):
        nv.simulate_mx("flat+e4m3", [np.zeros(64, np.float32)] * 9, "float32", pre=1.0)


def test_typed_program_dump_marks_wire_operands():
    d = nv.plan_dump("ring+f32", 0, 4, 4096, "bfloat16")
    assert "wire type fp32" in d and "STG~" in d
    d = nv.plan_dump("flat+pull+e4m3", 1, 4, 4096, "float32")
    assert "wire type e4m3" in d and "unit 1 B" in d


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("spec", ["flat+pull+e4m3", "flat+push+e4m3", "flat+pull+e5m2", "flat+pull+mxe4m3",
                                  "flat+push+mxe4m3"])
def test_fp8_wire_programs_sum_no_wire_only_operands(n, spec):
    """The fp8 / MX wire kernels carry the untyped path for wire-to-wire copies only (device_exec.hpp
    xfer_dispatch KM; planner.hpp typed_pattern_ok admits no other all-wire op for an fp8 wire): every planned
    fp8 program sums with the rank's own dtype value in the mix, and its widest fan-in is N (the kernel class)."""
    import re

    for rank in sorted({0, n - 1}):
        d = nv.plan_dump(spec, rank, n, 1 << 16, "bfloat16")
        widest = 0
        for line in d.splitlines():
            m = re.match(r"\s+XFER len=\d+ \[(.*)\] -> \[(.*)\]", line)
            if not m:
                continue
            srcs, dsts = m.group(1).split(" + "), m.group(2).split(", ")
            widest = max(widest, len(srcs))
            if len(srcs) >= 2:
                assert not all("~" in x for x in srcs + dsts), (spec, n, rank, line)
        assert widest == n, (spec, n, rank, widest)
