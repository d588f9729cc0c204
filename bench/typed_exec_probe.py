#!/usr/bin/env python3
"""Effective HBM rate of one executor schedule, typed or not: N ranks in one launch on one GPU (LocalGroup),
ITERS calls of SPEC on MIB MiB per rank, hipEvent-timed; the bytes are the program-cost model's (summed over
the ranks, csrc/include/flexar/cost_model.hpp program_cost, which matches rocprofv3 FETCH/WRITE counters:
profiles/r3_pmc_model). Run under `rocprofv3 --kernel-trace --stats` for per-kernel times.

    python3 bench/typed_exec_probe.py SPEC DTYPE       # SPEC "fp8" = all_reduce_fp8 (flat, e4m3 wire, AVG);
                                                       # "flat+pull+mxe4m3" = the OCP MX wire (AVG)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.parallel import LocalGroup

    spec, dtype = sys.argv[1], sys.argv[2]
    n = int(os.environ.get("TEP_RANKS", "4"))
    mib = int(os.environ.get("TEP_MIB", "100"))
    iters = int(os.environ.get("TEP_ITERS", "10"))
    dt = getattr(torch, dtype)
    count = (mib << 20) // dt.itemsize
    grp = LocalGroup(n, workspace_bytes=6 * (mib << 20) + (64 << 20))
    if os.environ.get("TEP_GRID"):  # workgroups per rank (a multiple of the program's channel count)
        grp.set_grid(int(os.environ["TEP_GRID"]))
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(count, device="cuda", generator=g).to(dt) for _ in range(n)]
    ys = [torch.empty_like(x) for x in xs]
    coll = os.environ.get("TEP_COLL", "all_reduce")
    if coll == "reduce_scatter":  # MIB per rank of input, MIB / N of output; "+mx..." specs: the MX wire
        m = count // n
        ins = [x[: n * m] for x in xs]
        outs = [torch.empty(m, device="cuda", dtype=dt) for _ in range(n)]
        op = "avg" if "+mx" in spec else "sum"
        run = lambda: grp.collective("reduce_scatter", ins, outs, op=op, algo=spec)  # noqa: E731
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            run()
        b.record()
        torch.cuda.synchronize()
        print(json.dumps({"coll": coll, "spec": spec, "dtype": dtype, "ranks": n, "mib_per_rank": mib,
                          "us_per_call": round(a.elapsed_time(b) * 1e3 / iters, 1)}), flush=True)
        grp.close()
        return
    if spec == "fp8":
        from allreduce_over_mpi_amd.ops.quant import fp8_amax

        parts = [fp8_amax(x) for x in xs]
        run = lambda: grp.all_reduce_fp8(xs, op="avg", outs=ys)  # noqa: E731
        model_spec = "flat+pull+e4m3"
        del parts
    else:  # "+mxe4m3" / "+mxe5m2": the OCP MX wire, no amax pass (AVG like the fp8 case)
        op = "avg" if "+mx" in spec else "sum"
        run = lambda: grp.all_reduce(xs, op, outs=ys, algo=spec)  # noqa: E731
        model_spec = spec
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        run()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / iters
    rd = wr = 0.0
    for r in range(n):
        c = nv.program_cost(model_spec, r, n, count, dtype, links=1)
        rd += c["hbm_read"]
        wr += c["hbm_write"]
    grp.check()
    print(json.dumps({"spec": spec, "dtype": dtype, "ranks": n, "mib_per_rank": mib, "us_per_call": round(us, 1),
                      "model_hbm_MiB": round((rd + wr) / 2**20, 1),
                      "effective_TBps": round((rd + wr) / (us * 1e-6) / 1e12, 3)}), flush=True)
    grp.close()


if __name__ == "__main__":
    main()
