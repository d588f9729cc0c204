#!/usr/bin/env python3
"""Measure every flexar algorithm across buffer sizes on THIS node and write a tune table.

The reference picks its topology offline with a closed-form cost model and a human exporting
FT_TOPO (cost_model/main.cpp, cost_model/CostModel.h:82-120). flexar's selector (cost_model.hpp)
models xGMI; this tool replaces the model with measurements: for each size (x4 steps) it validates
and times every candidate on all ranks (max over ranks), and writes the winners as FLEXAR_TUNE_FILE
lines "nranks bytes spec" (cost_model.hpp TuneTable: a row covers sizes >= bytes).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/flexar_tune.py --min-bytes 4K --max-bytes 1G --out tune_mi355x_8.txt
    FLEXAR_TUNE_FILE=tune_mi355x_8.txt python train.py ...

FLEXAR_BENCH_SHARED_GPU=1 rehearses it with every rank on device 0 (gloo bootstrap).

The same measurements calibrate the cost model: every run also fits the model's
(alpha_launch, alpha_sync, link_gbps, hbm_gbps) to the rows (utils/costfit.py) and prints FLEXAR_MODEL, and

    python tools/flexar_tune.py --fit rows.jsonl --nranks 4        # offline, no GPU

fits a saved --jsonl file.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_bytes(v: str) -> int:
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    v = v.strip().upper().rstrip("B")
    return int(float(v[:-1]) * mult[v[-1]]) if v and v[-1] in mult else int(float(v))


def candidates(world: int, nbytes: int) -> list[str]:
    from allreduce_over_mpi_amd.parallel.autotune import default_candidates

    return default_candidates(world, nbytes)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-bytes", default="4K")
    ap.add_argument("--max-bytes", default="256M")
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16", "float16"])
    ap.add_argument("--iters", type=int, default=0, help="timed calls per candidate (0 = by size)")
    ap.add_argument("--out", default="flexar_tune.txt")
    ap.add_argument("--jsonl", default="", help="also write every measurement as JSON lines")
    ap.add_argument("--fit", default="", help="offline: fit the cost model to this --jsonl file and exit")
    ap.add_argument("--nranks", type=int, default=0, help="--fit: world size of the rows (default: n_gpus field)")
    ap.add_argument("--links", type=int, default=0, help="--fit: concurrent links per GPU (0: the model default)")
    args = ap.parse_args()
    if args.fit:
        from allreduce_over_mpi_amd.utils.costfit import fit_model

        rows = [json.loads(line) for line in open(args.fit) if line.strip()]
        n = args.nranks or int(rows[0].get("n_gpus", 0))
        print(json.dumps(fit_model(rows, n, args.links)))
        return

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    shared = os.environ.get("FLEXAR_BENCH_SHARED_GPU", "0") == "1"
    local = 0 if shared else int(os.environ.get("LOCAL_RANK", "0"))
    if shared:
        os.environ.setdefault("FLEXAR_MAX_GRID", str(max(8, 256 // (2 * world))))
    os.environ.setdefault("FLEXAR_TIMEOUT_MS", "5000")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world < 2:
        raise SystemExit("flexar_tune needs >= 2 ranks (torch.distributed.run --nproc-per-node N)")
    dist.init_process_group("gloo" if shared else "nccl", **({} if shared else {"device_id": dev}))

    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.parallel import Communicator
    from allreduce_over_mpi_amd.utils.perf import busbw_gbps

    dtype = getattr(torch, args.dtype)
    es = torch.tensor([], dtype=dtype).element_size()
    lo, hi = parse_bytes(args.min_bytes), parse_bytes(args.max_bytes)
    ws = max(512 << 20, 2 * world * hi + (64 << 20))
    comm = Communicator(workspace_bytes=ws)

    def max_over_ranks(v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64, device="cpu" if shared else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    rows, table = [], []
    b = lo
    while b <= hi:
        n = max(1, b // es)
        g = torch.Generator(device=dev)
        g.manual_seed(17 + rank)
        x = torch.randn(n, device=dev, generator=g).to(dtype)
        y = torch.empty_like(x)
        ref = x.float().cpu()
        dist.all_reduce(ref)
        ref = ref.to(dev)
        iters = args.iters or max(5, min(200, int(5e8 // max(b, 1))))
        best, best_t = None, float("inf")
        for spec in candidates(world, n * es):
            # exactly two agreements per candidate on every rank whatever raised where (a rank whose check
            # raised must not skip a collective its peers make: theirs would pair with its next one)
            failed = 0.0
            t = 0.0
            try:
                # three calls on x, x/2, x/4 (exact scalings): a stale staging line from either of the two
                # previous calls (same or other parity half) changes the result
                tol = {torch.float32: 1e-5, torch.bfloat16: 2e-2, torch.float16: 4e-3}[dtype] * 4 * math.sqrt(world)
                for sc in (1.0, 0.5, 0.25):
                    xs = x if sc == 1.0 else (x.float() * sc).to(dtype)
                    comm.all_reduce(xs, out=y, algo=spec)
                    torch.cuda.synchronize()
                    err = float((y.float() - ref * sc).abs().max().item())
                    if err > tol * (float(ref.abs().max().item()) * sc + 1e-6):
                        failed = 1.0
                comm.check()
            except nv.FlexarError:
                failed = 1.0
            if max_over_ranks(failed) == 0.0:
                try:
                    for _ in range(3):
                        comm.all_reduce(x, out=y, algo=spec)
                    torch.cuda.synchronize()
                    dist.barrier()
                    t0 = time.perf_counter()
                    for _ in range(iters):
                        comm.all_reduce(x, out=y, algo=spec)
                    torch.cuda.synchronize()
                    t = (time.perf_counter() - t0) / iters
                    comm.check()
                except nv.FlexarError:
                    failed = 1.0
            else:
                failed = 1.0
            if max_over_ranks(failed) != 0.0:
                comm.close()
                torch.cuda.synchronize()
                comm = Communicator(workspace_bytes=ws)
                continue
            t = max_over_ranks(t)
            row = {"n_gpus": world, "bytes": n * es, "spec": spec, "us": round(t * 1e6, 2),
                   "busbw_GBps": round(busbw_gbps(n * es, t, world), 2)}
            rows.append(row)
            if t < best_t:
                best, best_t = spec, t
        if best is not None:
            table.append((n * es, best))
            if rank == 0:
                print(f"[tune] {n * es:>12d} B  best {best:14s} {best_t * 1e6:9.2f} us", flush=True)
        b *= 4
    if rank == 0:
        with open(args.out, "w") as f:
            f.write(f"# flexar tune table: {world} ranks, {args.dtype}, measured by tools/flexar_tune.py\n")
            prev = None
            for nbytes, spec in table:
                if spec != prev:  # a row covers every size up to the next row
                    f.write(f"{world} {nbytes} {spec}\n")
                    prev = spec
        if args.jsonl:
            with open(args.jsonl, "w") as f:
                for r in rows:
                    f.write(json.dumps(r) + "\n")
        from allreduce_over_mpi_amd.utils.costfit import fit_model

        try:
            fit = fit_model(rows, world, int(comm.topology().get("links", 0)))
            fit.pop("sizes")
        except ValueError as e:
            fit = {"error": str(e)}
        print(json.dumps({"tune_file": args.out, "rows": len(table), "model_fit": fit}), flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
