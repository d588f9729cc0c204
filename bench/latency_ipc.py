#!/usr/bin/env python3
"""Small-message latency of the production path (one process per rank, IPC-mapped
workspaces, no host synchronisation between calls) — with every rank on ONE GPU.

All ranks sharing device 0 exercises the real launch + flag/granule protocol
(kernels of different processes run concurrently on the GPU) but not xGMI, so
these numbers are the protocol + launch floor, not 8-GPU latencies.

    python bench/latency_ipc.py --nranks 2 --out gpurun_out/latency_ipc.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, sizes, algos, iters, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("FLEXAR_MAX_GRID", "16")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from allreduce_over_mpi_amd.parallel import Communicator

    comm = Communicator(workspace_bytes=64 << 20)
    rows = []
    for nbytes in sizes:
        n = max(1, nbytes // 4)
        x = torch.ones(n, device="cuda")
        y = torch.empty_like(x)
        for algo in algos:
            for _ in range(5):
                comm.all_reduce(x, out=y, algo=algo)
            torch.cuda.synchronize()
            dist.barrier()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(iters):
                comm.all_reduce(x, out=y, algo=algo)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / iters * 1e3
            ok = bool(torch.all(y == world).item())
            t = torch.tensor([us])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            rows.append({"nranks": world, "bytes": n * 4, "algo": algo, "us_per_call": round(float(t.item()), 2),
                         "correct": ok})
    comm.check()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, rows))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--algos", default="ll,oneshot,flat,ring")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch.multiprocessing as mp

    sizes = [4, 256, 4096, 65536, 262144, 1 << 20]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, args.nranks, port, sizes, args.algos.split(","), args.iters, q))
          for r in range(args.nranks)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=600) for _ in range(args.nranks))
    for p in ps:
        p.join(60)
    rows = res[0]
    for r in rows:
        print(json.dumps(r))
    if args.out:
        with open(args.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
