#!/usr/bin/env python3
"""Copy-engine allreduce: pipelined pieces (round 2) vs the serial per-piece schedule (FLEXAR_DMA_SERIAL=1,
round 1), N ranks in one process on one GPU (LocalGroup). A call is split into pieces by
FLEXAR_CHUNK_BYTES; with the pipeline the SDMA copies of piece k+1 overlap the reduce of piece k and the
all-gather copies of k overlap the reduce-scatter copies of k+1. One JSON line per (mode, chunk)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker():
    sys.path.insert(0, REPO)
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    n = int(os.environ.get("DMAB_RANKS", "4"))
    mib = int(os.environ.get("DMAB_MIB", "256"))
    count = (mib << 20) // 2
    grp = LocalGroup(n, workspace_bytes=1 << 30)
    xs = [torch.randn(count, device="cuda").to(torch.bfloat16) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    for _ in range(2):
        grp.all_reduce(xs, outs=ys, algo="dma")
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        grp.all_reduce(xs, outs=ys, algo="dma")
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    ref = torch.stack([x.float() for x in xs]).sum(0)
    err = ((ys[0].float() - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps({"ranks": n, "MiB_bf16": mib, "chunk_MiB": int(os.environ.get("FLEXAR_CHUNK_BYTES", "0")) >> 20,
                      "serial": os.environ.get("FLEXAR_DMA_SERIAL", "0") == "1", "ms": round(ms, 3),
                      "busbw_GBps": round(mib * 2**20 / (ms * 1e-3) * 2 * (n - 1) / n / 1e9, 1),
                      "max_rel_err": round(err, 5)}), flush=True)
    grp.close()


def main():
    for chunk in (0, 64, 16):
        for serial in ("1", "0"):
            env = dict(os.environ, FLEXAR_DMA_SERIAL=serial, FLEXAR_CHUNK_BYTES=str(chunk << 20))
            subprocess.run([sys.executable, os.path.abspath(__file__), "--worker"], env=env, check=True, timeout=240)


if __name__ == "__main__":
    worker() if "--worker" in sys.argv else main()
