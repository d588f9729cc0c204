#!/usr/bin/env python3
"""Typed executors with ONE PROCESS PER RANK (the production kernels exec_mx_kernel / exec_kernel, not the in-process
group kernel), all ranks on device 0: the A/B of the typed workgroup size (FLEXAR_TYPED_THREADS).

Each rank runs the case on MIB MiB, ITERS calls after a barrier, hipEvent-timed; the slowest rank's time is printed,
with the untyped flat fp32 on the same bytes as the control. Ranks share the GPU, so this prices kernels (HBM and
occupancy), not xGMI. Run under `rocprofv3 --kernel-trace --stats` for per-kernel times.

    python3 bench/typed_mp_probe.py [CASES...]     # CASES like fp8:bfloat16 mx:float32 flat:float32
    env: TMP_RANKS (4), TMP_MIB (100), TMP_ITERS (10), TMP_GRID (per-rank FLEXAR_MAX_GRID, default 256 / ranks)
"""
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, mib, iters, grid, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID=str(grid), FLEXAR_CALIB="0",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=6 * (mib << 20) + (64 << 20))
        out = []
        for case in cases:
            kind, dtype = case.split(":")
            dt = getattr(torch, dtype)
            count = (mib << 20) // dt.itemsize
            g = torch.Generator(device="cuda").manual_seed(1 + rank)
            x = torch.randn(count, device="cuda", generator=g).to(dt)
            y = torch.empty_like(x)
            if kind == "fp8":
                run = lambda: comm.all_reduce_fp8(x, op="avg", out=y)  # noqa: E731
            elif kind == "mx":
                run = lambda: comm.all_reduce(x, op="avg", out=y, algo="flat+pull+mxe4m3")  # noqa: E731
            else:
                run = lambda: comm.all_reduce(x, op="sum", out=y, algo="flat+pull")  # noqa: E731
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            dist.barrier()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(iters):
                run()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / iters
            t = torch.tensor([us], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            comm.check()
            out.append({"case": case, "us_per_call": round(float(t.item()), 1)})
            del x, y
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


def main():
    import torch.multiprocessing as mp

    cases = sys.argv[1:] or ["flat:float32", "fp8:bfloat16", "mx:float32"]
    world = int(os.environ.get("TMP_RANKS", "4"))
    mib = int(os.environ.get("TMP_MIB", "100"))
    iters = int(os.environ.get("TMP_ITERS", "10"))
    grid = int(os.environ.get("TMP_GRID", str(max(8, 256 // world))))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, mib, iters, grid, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, out, err = q.get(timeout=240)
            if err:
                raise SystemExit(f"rank {rank} failed:\n{err}")
            res[rank] = out
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    from allreduce_over_mpi_amd import _native as nv

    base = next((r["us_per_call"] for r in res[0] if r["case"] == "flat:float32"), None)
    for r in res[0]:
        r.update(ranks=world, mib_per_rank=mib, grid_per_rank=grid, lib=os.path.basename(os.path.dirname(os.environ.get("FLEXAR_LIB_PATH") or nv.lib_path())),
                 vs_flat_fp32=round(r["us_per_call"] / base, 3) if base else None)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
