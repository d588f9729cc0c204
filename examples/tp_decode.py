#!/usr/bin/env python3
"""Tensor-parallel decode step: a latency-bound allreduce per layer, eager vs one captured hipGraph.

Each rank holds a Megatron-style shard of an L-layer MLP stack (W1 split by columns, W2 by rows). A
token's step is, per layer: y = gelu(x @ W1_r) @ W2_r, then an allreduce of y (one hidden vector, 8 KiB
in bf16 at H=4096), then x += y. At batch 1 the allreduce and the launches dominate, not the GEMMs.

    python examples/tp_decode.py --nranks 2                 # all ranks on device 0 (1-GPU box)
    torchrun --nproc-per-node 8 examples/tp_decode.py       # one rank per GPU

Modes timed: ``eager`` (flexar LL allreduce per layer), ``graph`` (the whole step, GEMMs and
allreduces, captured once into a hipGraph and replayed), ``rccl`` (eager torch.distributed allreduce on
an RCCL group, for comparison; skipped when the ranks share one GPU). Every mode is checked against an
fp32 reference of the same step.
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


def run(rank, world, args, q=None):
    import torch
    import torch.distributed as dist

    shared = q is not None
    if shared:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(args.port))
        os.environ.setdefault("FLEXAR_MAX_GRID", "16")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group("nccl")
    from allreduce_over_mpi_amd.parallel import Communicator

    comm = Communicator(workspace_bytes=64 << 20)
    dev = torch.device("cuda", torch.cuda.current_device())
    H, L, F = args.hidden, args.layers, 4 * args.hidden // world
    g = torch.Generator().manual_seed(1234)  # identical full weights on every rank, then sharded
    W1 = [(torch.randn(H, 4 * H, generator=g) / H ** 0.5) for _ in range(L)]
    W2 = [(torch.randn(4 * H, H, generator=g) / (4 * H) ** 0.5) for _ in range(L)]
    w1 = [w[:, rank * F:(rank + 1) * F].to(dev, torch.bfloat16).contiguous() for w in W1]
    w2 = [w[rank * F:(rank + 1) * F, :].to(dev, torch.bfloat16).contiguous() for w in W2]
    x0 = torch.randn(1, H, generator=g)

    ref = x0.clone()
    for l in range(L):  # fp32 reference of one step
        ref = ref + torch.nn.functional.gelu(ref @ W1[l]) @ W2[l]

    x = torch.empty(1, H, device=dev, dtype=torch.bfloat16)
    y = torch.empty(1, H, device=dev, dtype=torch.bfloat16)

    def step(allreduce):
        for l in range(L):
            torch.matmul(torch.nn.functional.gelu(x @ w1[l]), w2[l], out=y)
            allreduce(y)
            x.add_(y)

    def flexar_ar(t):
        comm.all_reduce(t, algo=args.algo)

    results = {}

    def timed(name, fn):
        x.copy_(x0.to(dev, torch.bfloat16))
        fn()
        torch.cuda.synchronize()
        err = ((x.float().cpu() - ref).abs().max() / ref.abs().max()).item()
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        t = torch.tensor([dt])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        results[name] = {"us_per_step": round(float(t.item()) * 1e6, 1),
                         "us_per_layer": round(float(t.item()) * 1e6 / L, 2), "rel_err": round(err, 4)}

    timed("eager", lambda: step(flexar_ar))

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step(flexar_ar)  # plans built before capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        step(flexar_ar)
    timed("graph", graph.replay)

    if not shared:
        timed("rccl", lambda: step(lambda t: dist.all_reduce(t)))

    comm.check()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()
    row = {"nranks": world, "hidden": H, "layers": L, "algo": args.algo or "auto", "shared_gpu": shared, **results}
    if q is not None:
        q.put((rank, row))
    elif rank == 0:
        print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, default=0, help="spawn this many ranks on device 0 (no torchrun)")
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--algo", default=None, help="flexar spec (default: the selector, LL at this size)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    if args.nranks:
        import torch.multiprocessing as mp

        args.port = _port()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=run, args=(r, args.nranks, args, q)) for r in range(args.nranks)]
        for p in ps:
            p.start()
        rows = dict(q.get(timeout=600) for _ in range(args.nranks))
        for p in ps:
            p.join(60)
        print(json.dumps(rows[0]), flush=True)
        if args.out:
            with open(args.out, "a") as f:
                f.write(json.dumps(rows[0]) + "\n")
    else:
        run(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), args)


if __name__ == "__main__":
    main()
