#!/usr/bin/env python3
"""DDP training step, gradients allreduced four ways:

    python bench/ddp_step_bench.py                  # 2 processes sharing GPU 0 (rehearsal), gpt-small
    DDPB_RANKS=4 DDPB_MODES=pg,hook python bench/ddp_step_bench.py

- `pg`:     ``init_process_group("flexar")`` with its defaults: DDP's own reducer calls the flexar c10d
            backend, whose zero-copy probe agrees (gloo MIN) on registering each new bucket during the first
            calls and sweeps dead registrations every 16 calls;
- `pg_nozc`: the same with ``FLEXAR_PG_ZC=0`` (no probe, no sweeps: staging schedules only);
- `hook`:   a gloo process group plus ``flexar_allreduce_hook`` (FlexarHookState defaults: every bucket
            registered, "flat+zc+push");
- `fp8hook` / `mxhook`: the same with fp8 gradients on the wire (``flexar_fp8_compress_hook``: amax kernel +
            one launch; ``flexar_mxfp8_compress_hook``: OCP MX block scales, one launch);
- `nccl`:   RCCL (``init_process_group("nccl")``; the ranks share one GPU, so each gets its own
            NCCL_HOSTID and RCCL carries the bytes over loopback sockets - the step time is not an xGMI figure).

Each rank trains the same GPT (random init, synthetic tokens, bf16 autocast, fp32 gradients, 25 MB
buckets). One JSON line per mode: ms per step (max over ranks), tokens/s, and the HOST time per allreduce
call (perf_counter around the backend's allreduce / the hook; for `nccl` a hook that issues
``dist.all_reduce(async_op=True)``, i.e. what DDP's reducer does), so per-call host overhead such as the
zero-copy probe's blocking gloo rounds shows up separately from the device time.
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
        if mode == "pg_nozc":
            os.environ["FLEXAR_PG_ZC"] = "0"
        if mode in ("pg", "pg_nozc", "nccl"):  # RCCL for the backend's fallbacks / the nccl mode
            os.environ.update(NCCL_HOSTID=f"ddpb-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        import torch
        import torch.distributed as dist
        from torch.nn.parallel import DistributedDataParallel as DDP

        from allreduce_over_mpi_amd.models.gpt import GPT, PRESETS, synthetic_batch
        from allreduce_over_mpi_amd.parallel import backend as fb

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        host = {"calls": 0, "s": 0.0}
        if mode in ("pg", "pg_nozc"):
            orig = fb.FlexarProcessGroup.allreduce

            def timed_allreduce(self, *a, **k):
                t0 = time.perf_counter()
                try:
                    return orig(self, *a, **k)
                finally:
                    host["calls"] += 1
                    host["s"] += time.perf_counter() - t0

            fb.FlexarProcessGroup.allreduce = timed_allreduce
            dist.init_process_group("flexar", rank=rank, world_size=world)
        elif mode == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = PRESETS[os.environ.get("DDPB_MODEL", "gpt-small")]
        torch.manual_seed(0)
        model = GPT(cfg).to(dev)
        ddp = DDP(model, device_ids=[0], bucket_cap_mb=float(os.environ.get("DDPB_BUCKET_MB", "25")))
        state = None
        if mode == "hook":
            state = fb.FlexarHookState(algo=os.environ.get("DDPB_HOOK_ALGO") or None)

            def hook(st, bucket):
                t0 = time.perf_counter()
                fut = fb.flexar_allreduce_hook(st, bucket)
                host["calls"] += 1
                host["s"] += time.perf_counter() - t0
                return fut

            ddp.register_comm_hook(state, hook)
        elif mode in ("fp8hook", "mxhook"):  # compressed gradients: global-scale fp8 / OCP MX fp8 on the wire
            state = fb.FlexarHookState(algo=os.environ.get("DDPB_HOOK_ALGO") or None)
            base = fb.flexar_fp8_compress_hook if mode == "fp8hook" else fb.flexar_mxfp8_compress_hook

            def chook(st, bucket):
                t0 = time.perf_counter()
                fut = base(st, bucket)
                host["calls"] += 1
                host["s"] += time.perf_counter() - t0
                return fut

            ddp.register_comm_hook(state, chook)
        elif mode == "nccl":
            def nccl_hook(_, bucket):
                t0 = time.perf_counter()
                buf = bucket.buffer().div_(world)
                fut = dist.all_reduce(buf, async_op=True).get_future().then(lambda f: f.value()[0])
                host["calls"] += 1
                host["s"] += time.perf_counter() - t0
                return fut

            ddp.register_comm_hook(None, nccl_hook)
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
        host.update(calls=0, s=0.0)
        steps = int(os.environ.get("DDPB_STEPS", "10"))
        t0 = time.perf_counter()
        per_step = []
        for _ in range(steps):
            ts = time.perf_counter()
            loss = step()
            if os.environ.get("DDPB_STEP_SYNC") == "1":  # per-step times (diagnostics; serialises steps)
                torch.cuda.synchronize()
            per_step.append(round((time.perf_counter() - ts) * 1e3, 2))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt, host["s"] / max(1, host["calls"])], device=dev if mode == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, host_call = float(t[0]), float(t[1])
        params = sum(p.numel() for p in model.parameters())
        res = {"mode": mode, "model": os.environ.get("DDPB_MODEL", "gpt-small"), "params": params, "ranks": world,
               "ms_per_step": round(dt / steps * 1e3, 2), "tokens_per_s": round(steps * batch * cfg.seq * world / dt, 1),
               "allreduce_calls_per_step": round(host["calls"] / steps, 2),
               "host_us_per_allreduce": round(host_call * 1e6, 1), "loss": round(float(loss.item()), 4)}
        if os.environ.get("DDPB_STEP_SYNC") == "1":
            res["step_ms"] = per_step
        if state is not None:
            res["registrations"] = state.registrations
            res["deregistrations"] = state.deregistrations
        if mode in ("pg", "pg_nozc"):
            pg = dist.group.WORLD
            res["zc_registrations"] = pg.stats.get("zc_registrations", 0)
            res["fallback_calls"] = pg.stats.get("fallback", 0)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def main():
    import torch.multiprocessing as mp

    world = int(os.environ.get("DDPB_RANKS", "2"))
    # every rank shares one GPU: keep the processes' hardware queues resident; a cap, since the
    # GPU box exports HIP's default of 4 explicitly
    if world >= 4 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) > 2:
        os.environ["GPU_MAX_HW_QUEUES"] = "2"
    ctx = mp.get_context("spawn")
    for mode in os.environ.get("DDPB_MODES", "pg,pg_nozc,hook,nccl").split(","):
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
        print(json.dumps(sorted(res, key=lambda x: x[0])[0][1]), flush=True)


if __name__ == "__main__":
    main()
