#!/usr/bin/env python3
"""HBM traffic of the allreduce executor, for rocprofv3 counter runs: N ranks in ONE launch on one GPU
(LocalGroup), so every rank's loads and stores, local and "remote" (peer staging), hit this GPU's HBM.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -o run -- python3 bench/pmc_group.py
    python3 bench/pmc_group.py --expect            # bytes the schedules must move per call

Expected bytes per call (S = bytes per rank, N ranks, flat two-shot):
  flat+pull: reads  N * [(N-1)/N S (push IN blocks) + S (reduce: own block + N-1 landed blocks)
                         + (N-1)/N S (pull published blocks)]
             writes N * [(N-1)/N S (landed) + 2 S/N (OUT block + published block) + (N-1)/N S (OUT)]
  flat+push: reads  N * [(N-1)/N S + S + (N-1)/N S (copy-out of pushed blocks)]
             writes N * [(N-1)/N S + S/N + (N-1)/N S (multicast) + (N-1)/N S (copy-out)]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def expected(n, s):
    f = (n - 1) / n
    return {
        "flat+pull": {"read": n * (f * s + s + f * s), "write": n * (f * s + 2 * s / n + f * s)},
        "flat+push": {"read": n * (f * s + s + f * s), "write": n * (f * s + s / n + f * s + f * s)},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--specs", default="flat+pull,flat+push")
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--expect", action="store_true")
    args = ap.parse_args()
    s = args.mib << 20
    if args.expect:
        print(json.dumps({"ranks": args.ranks, "bytes_per_rank": s, "expected": expected(args.ranks, s)}))
        return
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    g = LocalGroup(args.ranks, workspace_bytes=4 * s + (64 << 20))  # one launch per call
    xs = [torch.randn(s // 4, device="cuda") for _ in range(args.ranks)]
    ys = [torch.empty_like(x) for x in xs]
    for spec in args.specs.split(","):
        for _ in range(args.calls):
            g.all_reduce(xs, outs=ys, algo=spec)
    torch.cuda.synchronize()
    g.check()
    g.close()
    print(json.dumps({"ranks": args.ranks, "bytes_per_rank": s, "specs": args.specs, "calls": args.calls}))


if __name__ == "__main__":
    main()
