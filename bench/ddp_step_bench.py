#!/usr/bin/env python3
"""DDP training step with gradients allreduced by flexar: the staging hook vs the zero-copy hook.

    python bench/ddp_step_bench.py                 # 2 processes sharing GPU 0 (rehearsal), gpt-small
    DDPB_RANKS=4 DDPB_MODEL=gpt-medium python bench/ddp_step_bench.py

Each rank trains the same GPT (random init, synthetic tokens) under DistributedDataParallel over a gloo
process group. The gradient buckets are reduced by `flexar_allreduce_hook`, in two modes:
- `hook`: the auto-selected schedule through the IPC staging workspace;
- `zchook`: every bucket is registered on first sight and reduced by "flat+zc+push", with no staging.

Both modes run overlapped with backward. One JSON line per mode gives ms per step and tokens/s. On one shared
GPU the allreduce competes with the other ranks' backward kernels for the same HBM, which is where fewer
HBM bytes per allreduce show up.
"""
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                          FLEXAR_MAX_GRID=str(max(8, 256 // (2 * world))), FLEXAR_TIMEOUT_MS="20000")
        import torch
        import torch.distributed as dist
        from torch.nn.parallel import DistributedDataParallel as DDP

        from allreduce_over_mpi_amd.models.gpt import GPT, PRESETS, synthetic_batch
        from allreduce_over_mpi_amd.parallel import backend as fb

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = PRESETS[os.environ.get("DDPB_MODEL", "gpt-small")]
        torch.manual_seed(0)
        model = GPT(cfg).to(dev)
        ddp = DDP(model, device_ids=[0], bucket_cap_mb=float(os.environ.get("DDPB_BUCKET_MB", "25")))
        state = fb.FlexarHookState(zero_copy=mode == "zchook")
        ddp.register_comm_hook(state, fb.flexar_allreduce_hook)
        opt = torch.optim.AdamW(ddp.parameters(), lr=3e-4)
        gen = torch.Generator().manual_seed(1000 + rank)
        batch = int(os.environ.get("DDPB_BATCH", "4"))

        def step():
            x, y = synthetic_batch(cfg, batch, gen, dev)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = ddp(x)
                loss = torch.nn.functional.cross_entropy(logits.reshape(-1, cfg.vocab).float(), y.reshape(-1))
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            return loss

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        steps = int(os.environ.get("DDPB_STEPS", "10"))
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        params = sum(p.numel() for p in model.parameters())
        res = {"mode": mode, "model": os.environ.get("DDPB_MODEL", "gpt-small"), "params": params, "ranks": world,
               "ms_per_step": round(dt / steps * 1e3, 2), "tokens_per_s": round(steps * batch * cfg.seq * world / dt, 1),
               "loss": round(float(loss.item()), 4), "hook_calls": state.calls,
               "zero_copy_buckets": len(state._bucket_regs),
               "registrations": state.registrations}
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def main():
    import torch.multiprocessing as mp

    world = int(os.environ.get("DDPB_RANKS", "2"))
    ctx = mp.get_context("spawn")
    for mode in ("hook", "zchook"):
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=worker, args=(r, world, port, mode, q)) for r in range(world)]
        for p in ps:
            p.start()
        res = [q.get(timeout=600) for _ in range(world)]
        for p in ps:
            p.join(60)
        for rank, r, tb in res:
            if tb:
                raise SystemExit(f"rank {rank} failed:\n{tb}")
        print(json.dumps(sorted(res)[0][1]), flush=True)


if __name__ == "__main__":
    main()
