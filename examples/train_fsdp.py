#!/usr/bin/env python3
"""Sharded data-parallel (FSDP2 ``fully_shard``) GPT training on the "flexar" backend.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_fsdp.py

Parameter all-gathers and gradient reduce-scatters run flexar's direct-exchange programs over xGMI
(``dist.all_gather_into_tensor`` / ``dist.reduce_scatter_tensor`` and their coalesced forms); the
remaining collectives go to RCCL. Data: synthetic token batches; weights: random init.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt-small")
    ap.add_argument("--batch", type=int, default=8, help="sequences per rank")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--backend", default="flexar", choices=["flexar", "nccl"])
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.fsdp import MixedPrecisionPolicy, fully_shard

    from allreduce_over_mpi_amd.models.gpt import GPT, PRESETS, synthetic_batch
    from allreduce_over_mpi_amd.parallel import backend as _fb  # noqa: F401  registers "flexar"

    local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()  # ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group(args.backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    mesh = init_device_mesh("cuda", (world,))
    cfg = PRESETS[args.model]
    torch.manual_seed(0)
    model = GPT(cfg).to(dev)
    mp = MixedPrecisionPolicy(param_dtype=torch.bfloat16, reduce_dtype=torch.float32)
    for blk in model.blocks:
        fully_shard(blk, mesh=mesh, mp_policy=mp)
    fully_shard(model, mesh=mesh, mp_policy=mp)
    opt = torch.optim.AdamW(model.parameters(), lr=3e-4)
    gen = torch.Generator().manual_seed(1000 + rank)

    def step():
        x, y = synthetic_batch(cfg, args.batch, gen, dev)
        loss = model.loss(x, y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({"backend": args.backend, "model": args.model, "world": world,
                          "tokens_per_s": round(args.steps * args.batch * cfg.seq * world / dt, 1),
                          "ms_per_step": round(dt / args.steps * 1e3, 2), "final_loss": round(float(loss.item()), 4)}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
