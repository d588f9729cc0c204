"""Aligned vs misaligned caller buffers through the executor: LocalGroup ranks on one
GPU, one launch per allreduce, views at +0 / +4 / +8 B (fp32) and +2 B (bf16). Prints one JSON line per
case with the device time per call (hipEvents over `--iters` calls after warm-up).

    python bench/misaligned_bench.py                              # unaligned 16-B vector path (default)
    FLEXAR_SCALAR_MISALIGNED=1 python bench/misaligned_bench.py   # round-3 policy: scalar on misalignment
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--mb", type=float, default=64.0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--specs", default="flat,ring,rhd")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = args.ranks
    grp = LocalGroup(n, workspace_bytes=max(256 << 20, int(args.mb * (1 << 20)) * 4 + (64 << 20)))
    policy = "scalar-on-misalignment" if os.environ.get("FLEXAR_SCALAR_MISALIGNED") == "1" else "vector-any-alignment"
    for dtype, offs in ((torch.float32, (0, 1, 2)), (torch.bfloat16, (0, 1))):
        es = torch.tensor([], dtype=dtype).element_size()
        count = int(args.mb * (1 << 20)) // es
        bufs = [torch.ones(count + 64, device=dev, dtype=dtype) for _ in range(n)]
        outs = [torch.empty(count + 64, device=dev, dtype=dtype) for _ in range(n)]
        for spec in args.specs.split(","):
            for off in offs:
                ins = [b[off:off + count] for b in bufs]
                os_ = [b[off:off + count] for b in outs]
                for _ in range(3):
                    grp.all_reduce(ins, "sum", outs=os_, algo=spec)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    grp.all_reduce(ins, "sum", outs=os_, algo=spec)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                ok = bool(torch.all(os_[0] == n).item())
                print(json.dumps({"policy": policy, "dtype": str(dtype).replace("torch.", ""), "spec": spec,
                                  "offset_bytes": off * es, "ranks": n, "mib": args.mb, "us_per_call": round(us, 2),
                                  "correct": ok}), flush=True)
    grp.check()
    grp.close()


if __name__ == "__main__":
    main()
