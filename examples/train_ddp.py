#!/usr/bin/env python3
"""Data-parallel GPT training with gradients allreduced by flexar.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_ddp.py --comm backend
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_ddp.py --comm hook
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_ddp.py --comm nccl   # RCCL baseline

--comm backend : process group "flexar" (dist.all_reduce -> flexar executor, rest -> RCCL)
--comm hook    : process group "nccl" + DDP comm hook routing gradient buckets through flexar
--comm fp8hook : the same hook with fp8 e4m3 gradients on the wire (flexar_fp8_compress_hook)
--comm mxhook  : OCP MX fp8 gradients, a scale per 32-element block, one launch (flexar_mxfp8_compress_hook)
--comm zchook  : the hook with zero-copy buckets (registered on first sight, "flat+zc+push": no staging)
Data: synthetic token batches; weights: random init (no network / checkpoints needed).
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
    ap.add_argument("--comm", default="backend", choices=["backend", "hook", "fp8hook", "mxhook", "zchook", "nccl"])
    ap.add_argument("--model", default="gpt-small")
    ap.add_argument("--batch", type=int, default=8, help="sequences per rank")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bf16", action="store_true", help="bf16 autocast (gradients stay fp32)")
    ap.add_argument("--bucket-mb", default="100",
                    help="DDP bucket size in MiB, or 'auto': the smallest bucket the calibrated selector prices at "
                         "90 %% of its 1 GiB bandwidth on this node (Communicator.recommended_bucket_bytes)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    from allreduce_over_mpi_amd.models.gpt import GPT, PRESETS, synthetic_batch
    from allreduce_over_mpi_amd.parallel import backend as fb

    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if int(os.environ.get("LOCAL_WORLD_SIZE", "1")) > ndev:  # more ranks than GPUs (a 1-GPU rehearsal)
        local %= ndev
        # RCCL refuses two ranks of one host on one GPU; a host id per rank makes it treat them as separate
        # hosts (loopback sockets), as bench.py's shared-GPU rehearsal does
        os.environ.setdefault("NCCL_HOSTID", f"train-ddp-rank{os.environ.get('RANK', '0')}")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("flexar" if args.comm == "backend" else "nccl")
    rank, world = dist.get_rank(), dist.get_world_size()
    cfg = PRESETS[args.model]
    torch.manual_seed(0)
    model = GPT(cfg).to(dev)
    if args.bucket_mb == "auto":
        from allreduce_over_mpi_amd.parallel import Communicator

        probe = Communicator(device=local)  # collective: connect, self-test, calibrated (or cached) model
        bucket_mb = probe.recommended_bucket_bytes(0.9, zero_copy=args.comm in ("backend", "zchook")) / 2**20
        probe.close()
    else:
        bucket_mb = float(args.bucket_mb)
    ddp = DDP(model, device_ids=[local], bucket_cap_mb=bucket_mb)
    if args.comm in ("hook", "fp8hook", "mxhook", "zchook"):
        hook = {"fp8hook": fb.flexar_fp8_compress_hook,
                "mxhook": fb.flexar_mxfp8_compress_hook}.get(args.comm, fb.flexar_allreduce_hook)
        ddp.register_comm_hook(fb.FlexarHookState(zero_copy=args.comm == "zchook"), hook)
    opt = torch.optim.AdamW(ddp.parameters(), lr=3e-4)
    gen = torch.Generator().manual_seed(1000 + rank)

    def step():
        x, y = synthetic_batch(cfg, args.batch, gen, dev)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.bf16):
            logits = ddp(x)
            loss = torch.nn.functional.cross_entropy(logits.reshape(-1, cfg.vocab).float(), y.reshape(-1))
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
    tokens = args.steps * args.batch * cfg.seq * world
    params = sum(p.numel() for p in model.parameters())
    if rank == 0:
        print(json.dumps({"comm": args.comm, "model": args.model, "params": params, "world": world,
                          "tokens_per_s": round(tokens / dt, 1), "ms_per_step": round(dt / args.steps * 1e3, 2),
                          "final_loss": round(float(loss.item()), 4), "bf16": args.bf16,
                          "bucket_mb": bucket_mb}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
