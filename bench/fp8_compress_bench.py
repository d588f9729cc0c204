#!/usr/bin/env python3
"""fp8 gradient compression on one MI355X: the fused kernels (ops/quant.py, one HBM pass each) against
the chain of PyTorch elementwise ops they replace, for DDP-sized buckets. Prints JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from allreduce_over_mpi_amd.ops import fp8_amax, fp8_dequantize, fp8_quantize

    dev = torch.device("cuda", 0)

    def t_of(fn, iters=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e3  # us

    num = 448.0 / 8
    for dtype in (torch.float32, torch.bfloat16):
        for mb in (25, 100):
            n = (mb << 20) // torch.tensor([], dtype=dtype).element_size()
            x = torch.randn(n, device=dev).to(dtype)
            out = torch.empty_like(x)

            def torch_chain():
                amax = x.abs().max().float().reshape(1)
                s = num / amax
                q = (x.float() * s).clamp(-448, 448).to(torch.float8_e4m3fn)
                out.copy_(q.float() / s)

            def fused():
                amax = fp8_amax(x)
                q = fp8_quantize(x, amax, num)
                fp8_dequantize(q, amax, num, out=out)

            tt, tf = t_of(torch_chain), t_of(fused)
            es = x.element_size()
            hbm = n * (es + es + 1 + 1 + es)  # amax read, quant read + write, dequant read + write
            print(json.dumps({"dtype": str(dtype).replace("torch.", ""), "MiB": mb, "torch_ops_us": round(tt, 1),
                              "fused_us": round(tf, 1), "speedup": round(tt / tf, 2),
                              "fused_hbm_TBps": round(hbm / (tf * 1e-6) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
