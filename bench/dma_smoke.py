#!/usr/bin/env python3
"""Minimal copy-engine (dma) allreduce check on one GPU with progress output (debug aid)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    for n in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2,3,4,8").split(",")]:
        g = LocalGroup(n, workspace_bytes=64 << 20)
        for size in (1, 35, 1000, 65539, (1 << 20) + 5):
            xs = [torch.full((size,), float(r + 1), device="cuda") for r in range(n)]
            for it in range(3):
                t = time.perf_counter()
                ys = g.all_reduce([x.clone() for x in xs], algo="dma")
                torch.cuda.synchronize()
                ok = all(bool(torch.all(y == n * (n + 1) / 2).item()) for y in ys)
                print(f"n={n} size={size} it={it} ok={ok} {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
                try:
                    g.check()
                except Exception as e:  # noqa: BLE001 - report and continue to the next size
                    print("  check:", e, flush=True)
        g.close()


if __name__ == "__main__":
    main()
