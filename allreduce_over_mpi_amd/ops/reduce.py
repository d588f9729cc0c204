"""Standalone gfx950 reduction kernel: ``out = scale * OP(srcs)``.

The MI355X counterpart of the reference's CPU ``reduce_sum`` / ``reduce_band``
(allreduce_over_mpi/mpi_mod.hpp:245-660): one vectorised HIP kernel
(16 B per lane, fp32 accumulation for bf16/fp16/fp8, fused scale) instead of
a hand-unrolled OpenMP loop per fan-in. Fan-in 1..64 (chained in groups of 8).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

from .. import _native as nv


def reduce(srcs: Sequence, op="sum", scale: float = 1.0, out=None, stream=None):
    import torch

    if not srcs:
        raise nv.FlexarError(1, "need at least one source")
    t0 = srcs[0]
    for s in srcs:
        if not s.is_cuda or not s.is_contiguous() or s.dtype != t0.dtype or s.numel() != t0.numel():
            raise nv.FlexarError(1, "sources must be contiguous device tensors of one dtype and size")
    if out is None:
        out = torch.empty_like(t0)
    arr = (ctypes.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    st = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
    nv.check(nv.lib().flexar_reduce(out.data_ptr(), arr, len(srcs), t0.numel(), nv.dtype_code(t0.dtype),
                                    nv.op_code(op), float(scale), st), "reduce")
    return out


def reduce_host(srcs: Sequence, op="sum", scale: float = 1.0, dtype: Optional[str] = None):
    """Host (CPU) reduction used by the MPI/shared-memory plumbing path (numpy arrays)."""
    return nv.reduce_host(srcs, op=op, scale=scale, dtype=dtype)
