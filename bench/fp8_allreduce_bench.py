#!/usr/bin/env python3
"""fp8-compressed allreduce on one MI355X (BASELINE config #5): the round-2 fused path against the round-1
launch chain, N ranks in one process on one GPU (LocalGroup: every rank's workgroups in one launch).

  chain  (round 1): amax, MAX allreduce of the partials (LL), quantize, fp8 allreduce (+1/N), dequantize
                    = 3 per-rank elementwise passes + 2 allreduce launches
  fused  (round 2): amax, ONE allreduce launch that exchanges the amax, quantises inside the first
                    transfer and dequantises inside the last (Communicator.all_reduce_fp8)
  plain:            the uncompressed flat allreduce of the same buffer (dtype on the wire)

With every rank on one GPU the "links" are the shared HBM, so this prices launches and HBM passes, not
xGMI time. Prints JSON lines (device time per call from hipEvents)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from allreduce_over_mpi_amd.ops import fp8_amax, fp8_dequantize, fp8_quantize
    from allreduce_over_mpi_amd.parallel import LocalGroup

    n = int(os.environ.get("FP8B_RANKS", "4"))
    sizes = [int(v) for v in os.environ.get("FP8B_MIB", "25,100").split(",")]
    iters = int(os.environ.get("FP8B_ITERS", "20"))
    dev = torch.device("cuda", 0)
    grp = LocalGroup(n, workspace_bytes=640 << 20)

    def t_of(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e3  # us per call (all ranks)

    for dtype in (torch.float32, torch.bfloat16):
        for mb in sizes:
            count = (mb << 20) // torch.tensor([], dtype=dtype).element_size()
            g = torch.Generator(device=dev).manual_seed(mb)
            xs = [torch.randn(count, device=dev, generator=g).to(dtype) for _ in range(n)]
            ys = [torch.empty_like(x) for x in xs]
            num = 448.0 / n

            def chain():
                parts = [fp8_amax(x) for x in xs]
                grp.all_reduce(parts, "max")
                qs = [fp8_quantize(x, p, num) for x, p in zip(xs, parts)]
                grp.all_reduce(qs, "avg", algo="flat")
                for q, p, y in zip(qs, parts, ys):
                    fp8_dequantize(q, p, num, out=y)

            def fused():
                grp.all_reduce_fp8(xs, op="avg", outs=ys)

            def plain():
                grp.all_reduce(xs, "avg", outs=ys, algo="flat")

            t_chain, t_fused, t_plain = t_of(chain), t_of(fused), t_of(plain)
            ref = torch.stack([x.double() for x in xs]).mean(0)
            fused()
            torch.cuda.synchronize()
            err = ((ys[0].double() - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"ranks": n, "dtype": str(dtype).replace("torch.", ""), "MiB_per_rank": mb,
                              "chain_us": round(t_chain, 1), "fused_us": round(t_fused, 1),
                              "plain_us": round(t_plain, 1), "fused_vs_chain": round(t_chain / t_fused, 2),
                              "launches_chain": 3 * n + 2 + n, "launches_fused": n + 1,
                              "fused_max_rel_err": round(err, 4)}), flush=True)
    grp.close()


if __name__ == "__main__":
    main()
