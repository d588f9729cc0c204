#!/usr/bin/env python3
"""Expert-parallel MoE token dispatch / combine with equal-capacity all-to-all on the "flexar" backend.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/moe_dispatch.py
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/moe_dispatch.py --zero-copy

Every rank hosts one expert. Tokens are routed top-1 with a fixed capacity per (source rank, expert),
so dispatch and combine are equal-split ``dist.all_to_all_single`` calls, which flexar runs as one
direct exchange over all xGMI links. With ``--zero-copy`` the receive buffers are registered once with a
flexar Communicator and every rank writes its tokens straight into the peers' buffers (no staging). The
result is checked against running every expert locally.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse

    import torch
    import torch.distributed as dist

    ap = argparse.ArgumentParser()
    ap.add_argument("--zero-copy", action="store_true", help="registered receive buffers, zero-copy all-to-all")
    args = ap.parse_args()

    from allreduce_over_mpi_amd.parallel import backend as _fb  # noqa: F401

    local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()  # ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("flexar")
    rank, world = dist.get_rank(), dist.get_world_size()
    d, cap, tokens = 256, 64, 512
    torch.manual_seed(0)
    experts = [torch.nn.Linear(d, d).to(dev) for _ in range(world)]  # identical on every rank
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    x = torch.randn(tokens, d, device=dev, generator=g)
    route = torch.randint(0, world, (tokens,), device=dev, generator=g)

    # pack: slot [e, c] holds the c-th token this rank routes to expert e (capacity-dropped beyond cap)
    send = torch.zeros(world, cap, d, device=dev)
    kept = torch.zeros(world, cap, dtype=torch.long, device=dev) - 1
    for e in range(world):
        idx = (route == e).nonzero().flatten()[:cap]
        send[e, :len(idx)] = x[idx]
        kept[e, :len(idx)] = idx
    recv = torch.empty_like(send)
    back = torch.empty_like(send)
    if args.zero_copy:  # persistent dispatch / combine buffers, registered once (collective)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator()
        comm.register_many([recv, back])
        a2a = lambda out, inp: comm.all_to_all(inp, out)  # noqa: E731 - registered out: zero copy
    else:
        a2a = lambda out, inp: dist.all_to_all_single(out, inp)  # noqa: E731
    a2a(recv.view(-1), send.view(-1))                              # dispatch
    with torch.no_grad():
        out = experts[rank](recv.view(-1, d)).view(world, cap, d)  # this rank's expert on every source
    a2a(back.view(-1), out.contiguous().view(-1))                  # combine
    y = torch.zeros_like(x)
    with torch.no_grad():
        for e in range(world):
            m = kept[e] >= 0
            y[kept[e][m]] = back[e][m]
            ref = experts[e](x[kept[e][m]])
            assert torch.allclose(back[e][m], ref, atol=1e-4), "all-to-all dispatch/combine mismatch"
    if rank == 0:
        print(f"moe dispatch/combine ok: {world} experts, capacity {cap}, d={d}, zero copy {args.zero_copy}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
