"""fp8 (OCP e4m3) gradient compression kernels (csrc/src/k_quant.hip): one HBM pass each.

    parts = fp8_amax(x)                    # FLEXAR_AMAX_PARTIALS per-workgroup max |x| (device, no host sync)
    q = fp8_quantize(x, parts, num)        # e4m3(clamp(x * num / amax, +-448)), amax = parts.max()
    fp8_dequantize(q, parts, num, out=x)   # x = q * amax / num

Used by the fp8-compressed DDP hook (parallel/backend.py) between a MAX allreduce of the partials
(1 KiB) and the fp8 allreduce with the fused 1/N post-scale (BASELINE config #5).
"""
from __future__ import annotations

from .. import _native as nv
from ..parallel.comm import _stream_handle


def _check(t, what):
    if not t.is_cuda or not t.is_contiguous():
        raise nv.FlexarError(1, f"{what} must be a contiguous ROCm tensor")
    if t.data_ptr() % 16:
        raise nv.FlexarError(1, f"{what} must be 16-byte aligned")


AMAX_PARTIALS = 256  # FLEXAR_AMAX_PARTIALS


def fp8_amax(x, out=None, stream=None):
    import torch

    _check(x, "x")
    out = torch.empty(AMAX_PARTIALS, dtype=torch.float32, device=x.device) if out is None else out
    if out.numel() != AMAX_PARTIALS or out.dtype != torch.float32:
        raise nv.FlexarError(1, f"amax partials must be {AMAX_PARTIALS} float32 values")
    nv.check(nv.lib().flexar_amax(x.data_ptr(), x.numel(), nv.dtype_code(x.dtype), out.data_ptr(),
                                  _stream_handle(stream)), "amax")
    return out


def fp8_quantize(x, amax, num: float = 448.0, out=None, stream=None):
    import torch

    _check(x, "x")
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device) if out is None else out
    _check(q, "out")
    nv.check(nv.lib().flexar_quantize_fp8(x.data_ptr(), nv.dtype_code(x.dtype), q.data_ptr(), x.numel(),
                                          amax.data_ptr(), float(num), _stream_handle(stream)), "quantize_fp8")
    return q


def fp8_dequantize(q, amax, num: float = 448.0, out=None, dtype=None, stream=None):
    import torch

    _check(q, "q")
    x = torch.empty(q.shape, dtype=dtype or torch.float32, device=q.device) if out is None else out
    _check(x, "out")
    nv.check(nv.lib().flexar_dequantize_fp8(q.data_ptr(), x.data_ptr(), nv.dtype_code(x.dtype), q.numel(),
                                            amax.data_ptr(), float(num), _stream_handle(stream)), "dequantize_fp8")
    return x


def fp8_wire_scale(nranks: int, amax: float, wire: str = "e4m3") -> float:
    """The pre-scale s the fp8-wire executor derives on the device (device_exec.hpp fp8_scale): fp8_max /
    (N * global amax * (1 + h)), h the wire type's largest relative rounding step, computed in fp32 and
    rounded DOWN to a power of two (so x * s is exact and gfx950's scaled converts apply it). Every
    contribution is quantised as fp8(x * s) and the result written as q / s."""
    import numpy as np

    f = np.float32
    wmax, head = (f(448.0), f(1.0625)) if wire == "e4m3" else (f(57344.0), f(1.125))
    g = f(amax)
    s = wmax / (f(nranks) * g * head) if (g > 0 and g < f(3.0e38)) else f(1.0)
    s = min(max(s, f(2.0 ** -120)), f(2.0 ** 120))
    bits = np.array([s], dtype=np.float32).view(np.uint32)[0] & np.uint32(0x7F800000)
    return float(np.array([bits], dtype=np.uint32).view(np.float32)[0])


# ---- OCP MX block-scaled fp8 wire ("+mxe4m3" / "+mxe5m2", docs/DESIGN.md §9.2) --------------------------
MX_BLOCK = 32
_MX_EMAX = {"e4m3": 8, "e5m2": 15}


def mx_scale_bytes(x, wire: str = "e4m3"):
    """e8m0 scale byte of every 32-element block of the fp32 tensor ``x`` (1-D, any length; the last block may
    be partial) - types.hpp mx_scale_byte: 2^X with X the smallest exponent such that max|x| <= fp8_max * 2^X,
    as X + 127 clamped to [1, 254]. The maximum is taken over sign-cleared f32 bits (NaN / inf count as largest)."""
    import torch

    n = x.numel()
    pad = (-n) % MX_BLOCK
    bits = x.float().contiguous().view(torch.int32).to(torch.int64) & 0x7FFFFFFF
    if pad:
        bits = torch.cat([bits, torch.zeros(pad, dtype=torch.int64, device=bits.device)])
    am = bits.view(-1, MX_BLOCK).amax(1)
    e = (am >> 23) - _MX_EMAX[wire] + ((am & 0x7FFFFF) > 0x600000).to(torch.int64)
    return e.clamp(1, 254)


def mx_quantize(x, wire: str = "e4m3"):
    """(q, scale bytes): the fp8 values q = rne(x / 2^X) of every block of the fp32 tensor ``x`` and the blocks'
    e8m0 bytes - what the MX executor puts on the wire. Works on CPU and ROCm tensors (torch ops: the
    hierarchical communicator's cross-node compression uses it on the device)."""
    import torch

    sb = mx_scale_bytes(x, wire)
    sc = torch.pow(2.0, (sb - 127).double()).float().repeat_interleave(MX_BLOCK)[: x.numel()]
    fp8 = torch.float8_e4m3fn if wire == "e4m3" else torch.float8_e5m2
    return (x.float() / sc).to(fp8), sb


def mx_round(x, wire: str = "e4m3"):
    """x rounded through the MX wire: q * 2^X per block, fp32."""
    import torch

    q, sb = mx_quantize(x, wire)
    sc = torch.pow(2.0, (sb - 127).double()).float().repeat_interleave(MX_BLOCK)[: x.numel()]
    return q.float() * sc


def mx_allreduce_reference(inputs, wire: str = "e4m3", op: str = "sum"):
    """What the flat MX-wire allreduce computes (device_exec.hpp xfer_mxb, host_exec.hpp host_xfer_mxb), on CPU
    tensors of one float dtype: the count splits into N chunks of whole 256-element granules; the owner c of
    chunk c sums its own contribution and those of ranks c+1, c+2, ... (mod N) in fp32 - each rounded through
    MX with its sender's block scales - applies AVG's 1/N, rounds the sum through MX (the result's own block
    scales) and every rank gets that value in the input dtype."""
    import torch

    n = len(inputs)
    dt = inputs[0].dtype
    count = inputs[0].numel()
    split = (-(-count // n) + 255) // 256 * 256
    out = torch.empty(count, dtype=torch.float32)
    for c in range(n):
        lo, hi = min(count, c * split), min(count, (c + 1) * split)
        if hi <= lo:
            continue
        acc = None
        for k in range(n):
            src = (c + k) % n
            v = mx_round(inputs[src].reshape(-1)[lo:hi].float(), wire)
            acc = v if acc is None else acc + v
        if op == "avg":
            acc = acc * torch.tensor(1.0 / n, dtype=torch.float32)
        out[lo:hi] = mx_round(acc, wire)
    return out.to(dt)


def mx_reduce_scatter_reference(inputs, wire: str = "e4m3", op: str = "sum"):
    """What the flat reduce-scatter with the MX wire computes (planner.hpp build_flat_rs, "+mxe4m3"): rank r owns
    block r (count / N elements) of every input; it sums its own block and then ranks 0, 1, ... (without r),
    each rounded through MX with its sender's block scales (32-element blocks from the start of block r), in
    fp32, applies AVG's 1/N and writes the result in the input dtype (no second MX rounding: nothing of the
    result crosses a link)."""
    import torch

    n = len(inputs)
    dt = inputs[0].dtype
    m = inputs[0].numel() // n
    outs = []
    for r in range(n):
        order = [r] + [p for p in range(n) if p != r]
        acc = None
        for p in order:
            v = mx_round(inputs[p].reshape(-1)[r * m:(r + 1) * m].float(), wire)
            acc = v if acc is None else acc + v
        if op == "avg":
            acc = acc * torch.tensor(1.0 / n, dtype=torch.float32)
        outs.append(acc.to(dt))
    return outs


def mx_dequantize(q, scale_bytes, numel: int):
    """fp32 values q * 2^X of an MX payload (``q`` float8, ``scale_bytes`` one e8m0 byte per 32 elements)."""
    import torch

    sc = torch.pow(2.0, (scale_bytes.to(torch.int64) - 127).double()).float().repeat_interleave(MX_BLOCK)[:numel]
    return q.float() * sc


_MX_WIRE_CODES = {"e4m3": 4, "e5m2": 5}


def mx_message_bytes(n: int) -> int:
    """Bytes of an MX message of ``n`` elements: the fp8 values, then one scale byte per 32-element block."""
    return n + (n + MX_BLOCK - 1) // MX_BLOCK


def mx_pack(x, wire: str = "e4m3", out=None, stream=None):
    """Native MX codec (csrc/src/k_mx_codec.hip): the uint8 message [q | scale bytes] of the contiguous
    f32 / bf16 / f16 ROCm tensor ``x`` in one HBM pass - bitwise ``mx_quantize`` (fp8 bytes, then the scale
    bytes)."""
    import torch

    if not x.is_cuda or not x.is_contiguous():
        raise nv.FlexarError(1, "x must be a contiguous ROCm tensor")
    n = x.numel()
    msg = torch.empty(mx_message_bytes(n), dtype=torch.uint8, device=x.device) if out is None else out
    if msg.numel() < mx_message_bytes(n) or msg.dtype != torch.uint8 or not msg.is_contiguous():
        raise nv.FlexarError(1, "mx_pack: out must be contiguous uint8 of mx_message_bytes(n)")
    nv.check(nv.lib().flexar_mx_pack(x.data_ptr(), nv.dtype_code(x.dtype), msg.data_ptr(), n,
                                     _MX_WIRE_CODES[wire], _stream_handle(stream)), "mx_pack")
    return msg


def mx_unpack_sum(msgs, n: int, wire: str = "e4m3", out=None, stream=None, post: float = 1.0):
    """Sum of the dequantised MX messages ``msgs`` (uint8 [k, >= mx_message_bytes(n)], contiguous) in row
    order, fp32, in one pass (csrc/src/k_mx_codec.hip) - bitwise ``mx_dequantize`` of each row summed in
    order, times ``post`` (AVG's 1 / world fused into the same pass; 1 = none)."""
    import torch

    if not msgs.is_cuda or msgs.dim() != 2 or msgs.dtype != torch.uint8 or not msgs.is_contiguous():
        raise nv.FlexarError(1, "msgs must be a contiguous 2-D uint8 ROCm tensor")
    y = torch.empty(n, dtype=torch.float32, device=msgs.device) if out is None else out
    if y.dtype != torch.float32 or y.numel() != n or not y.is_contiguous():
        raise nv.FlexarError(1, "mx_unpack_sum: out must be contiguous float32 of n elements")
    nv.check(nv.lib().flexar_mx_unpack_sum_scaled(msgs.data_ptr(), msgs.shape[1], msgs.shape[0], n,
                                                  _MX_WIRE_CODES[wire], float(post), y.data_ptr(),
                                                  _stream_handle(stream)), "mx_unpack_sum")
    return y
