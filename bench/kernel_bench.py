#!/usr/bin/env python3
"""Single-GPU microbenchmarks of the flexar kernels (one MI355X).

1. ``reduce``: the standalone reduction kernel, fan-in K, dtypes f32/bf16/fp8 —
   effective HBM bandwidth = (K reads + 1 write) bytes / time (roofline: HBM).
2. ``group``: the full allreduce protocol with N ranks in ONE launch on one GPU
   (LocalGroup). Peers' staging is local HBM here, so this measures the
   executor's protocol overhead (flags, epochs, slicing) and small-message
   latency floors, not xGMI bandwidth.
3. ``copy``: the N=1 allreduce path (out-of-place copy through the executor).

Writes one JSON line per measurement to stdout (and --out file).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warm=3):
    import torch

    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="reduce,group,copy")
    ap.add_argument("--out", default="")
    ap.add_argument("--reduce-mb", type=float, default=256)
    ap.add_argument("--dtypes", default="float32,bfloat16,float8_e4m3fn")
    ap.add_argument("--fanins", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    from allreduce_over_mpi_amd.ops import reduce
    from allreduce_over_mpi_amd.parallel import Communicator, LocalGroup

    dev = torch.device("cuda", 0)
    rows = []

    def emit(**kw):
        rows.append(kw)
        print(json.dumps(kw), flush=True)

    what = set(args.what.split(","))
    if "reduce" in what:
        for dt in [getattr(torch, d) for d in args.dtypes.split(",")]:
            es = torch.tensor([], dtype=dt).element_size()
            n = int(args.reduce_mb * (1 << 20)) // es
            for k in [int(f) for f in args.fanins.split(",")]:
                srcs = [torch.randn(n, device=dev).to(dt) for _ in range(k)]
                out = torch.empty_like(srcs[0])
                t = timeit(lambda: reduce(srcs, "sum", out=out), iters=args.iters)
                emit(kind="reduce", dtype=str(dt).replace("torch.", ""), fanin=k, bytes_per_src=n * es,
                     us=round(t * 1e6, 2), eff_TBps=round((k + 1) * n * es / t / 1e12, 3))
                del srcs, out
                torch.cuda.empty_cache()
    if "copy" in what:
        c = Communicator(rank=0, world_size=1, workspace_bytes=16 << 20)
        for mb in (1, 16, 256, 1024):
            n = (mb << 20) // 4
            x = torch.randn(n, device=dev)
            y = torch.empty_like(x)
            t = timeit(lambda: c.all_reduce(x, out=y))
            emit(kind="copy", MiB=mb, us=round(t * 1e6, 2), algbw_GBps=round(n * 4 / t / 1e9, 1),
                 hbm_TBps=round(2 * n * 4 / t / 1e12, 3))
        c.close()
    if "group" in what:
        for nr in (2, 4, 8):
            g = LocalGroup(nr, workspace_bytes=640 << 20)
            specs = ["oneshot", "flat+pull", "flat+push", "ring", "ring:4" if nr >= 4 else "ring:2"]
            if nr == 8:
                specs += ["rhd+pull", "tree:2,4+push"]
            for kib in (4, 64, 1024, 16384, 262144):
                n = kib * 1024 // 4
                xs = [torch.randn(n, device=dev) for _ in range(nr)]
                ys = [torch.empty_like(x) for x in xs]
                for spec in specs:
                    if spec == "oneshot" and kib > 16384:
                        continue
                    try:
                        t = timeit(lambda: g.all_reduce(xs, outs=ys, algo=spec), iters=10, warm=2)
                    except Exception as e:  # noqa: BLE001
                        emit(kind="group", nranks=nr, KiB=kib, algo=spec, error=str(e)[:200])
                        continue
                    emit(kind="group", nranks=nr, KiB=kib, algo=spec, us=round(t * 1e6, 2),
                         busbw_GBps_1gpu=round(n * 4 / t / 1e9 * 2 * (nr - 1) / nr, 1))
            g.check()
            g.close()
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
