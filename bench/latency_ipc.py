#!/usr/bin/env python3
"""Small-message latency of the production path (one process per rank, IPC-mapped
workspaces, no host synchronisation between calls) — with every rank on ONE GPU.

All ranks sharing device 0 exercises the real launch + flag/granule protocol
(kernels of different processes run concurrently on the GPU) but not xGMI, so
these numbers are the protocol + launch floor, not 8-GPU latencies.

    python bench/latency_ipc.py --nranks 2 --out gpurun_out/latency_ipc.jsonl
    python bench/latency_ipc.py --nranks 2 --graph      # the same calls captured in one hipGraph
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, sizes, algos, iters, q, graph=False):
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
            if graph:
                # launch-bound loop as one hipGraph: `iters` allreduces captured once, replayed; per-call
                # cost is the protocol without the host launch path
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(iters):
                        comm.all_reduce(x, out=y, algo=algo)
                torch.cuda.current_stream().wait_stream(s)
                for _ in range(2):
                    g.replay()
                torch.cuda.synchronize()
                dist.barrier()
                a.record()
                h0 = time.perf_counter()
                g.replay()
                h1 = time.perf_counter()
                b.record()
            else:
                a.record()
                h0 = time.perf_counter()
                for _ in range(iters):
                    comm.all_reduce(x, out=y, algo=algo)
                h1 = time.perf_counter()
                b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / iters * 1e3
            host_us = (h1 - h0) / iters * 1e6  # CPU time to issue one call (eager) / 1/iters of a replay
            ok = bool(torch.all(y == world).item())
            t = torch.tensor([us, host_us])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            rows.append({"nranks": world, "bytes": n * 4, "algo": algo, "us_per_call": round(float(t[0]), 2),
                         "host_us_per_call": round(float(t[1]), 2), "correct": ok, "graph": graph})
        # floor: the same number of back-to-back single-kernel torch launches (a device copy)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            y.copy_(x)
        torch.cuda.synchronize()
        a.record()
        h0 = time.perf_counter()
        for _ in range(iters):
            y.copy_(x)
        h1 = time.perf_counter()
        b.record()
        torch.cuda.synchronize()
        t = torch.tensor([a.elapsed_time(b) / iters * 1e3, (h1 - h0) / iters * 1e6])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        rows.append({"nranks": world, "bytes": n * 4, "algo": "torch_copy_floor", "us_per_call": round(float(t[0]), 2),
                     "host_us_per_call": round(float(t[1]), 2), "correct": True, "graph": False})
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
    ap.add_argument("--sizes", default="4,256,4096,65536,262144,1048576", help="buffer bytes")
    ap.add_argument("--graph", action="store_true", help="capture the timed calls in one hipGraph and replay it")
    args = ap.parse_args()
    import torch.multiprocessing as mp

    sizes = [int(v) for v in args.sizes.split(",")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, args.nranks, port, sizes, args.algos.split(","), args.iters, q, args.graph))
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
