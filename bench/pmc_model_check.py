#!/usr/bin/env python3
"""Program-cost model vs rocprofv3 HBM counters ("price schedules from the compiled
program"): N ranks in ONE launch on one GPU (LocalGroup), so every rank's loads and stores - local and
"remote" - hit this GPU's HBM, and FETCH_SIZE / WRITE_SIZE per dispatch can be set against the bytes the
model reads off the programs (csrc/include/flexar/cost_model.hpp program_cost, summed over the ranks).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- python3 bench/pmc_model_check.py SPEC DTYPE
    python3 bench/pmc_model_check.py --predict SPEC DTYPE      # the model's bytes per dispatch (JSON)

SPEC "fp8" = all_reduce_fp8 (flat, e4m3 wire, AVG), priced as "flat+pull+e4m3" (the amax kernel is a
separate dispatch and not counted).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

RANKS = int(os.environ.get("PMC_RANKS", "4"))
MIB = int(os.environ.get("PMC_MIB", "64"))


def predict(spec, dtype):
    from allreduce_over_mpi_amd import _native as nv

    es = {"float32": 4, "bfloat16": 2}[dtype]
    n = (MIB << 20) // es
    tot = {"read": 0.0, "write": 0.0}
    model_spec = "flat+pull+e4m3" if spec == "fp8" else spec
    for r in range(RANKS):
        c = nv.program_cost(model_spec, r, RANKS, n, dtype, links=1)
        tot["read"] += c["hbm_read"]
        tot["write"] += c["hbm_write"]
    return {"spec": spec, "dtype": dtype, "ranks": RANKS, "mib_per_rank": MIB, "read_MiB": tot["read"] / 2**20,
            "write_MiB": tot["write"] / 2**20}


def run(spec, dtype):
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    dt = getattr(torch, dtype)
    s = MIB << 20
    g = LocalGroup(RANKS, workspace_bytes=6 * s + (64 << 20))  # one launch per call
    xs = [torch.randn(s // dt.itemsize, device="cuda").to(dt) for _ in range(RANKS)]
    ys = [torch.empty_like(x) for x in xs]
    for _ in range(3):
        if spec == "fp8":
            g.all_reduce_fp8(xs, op="avg", outs=ys)
        else:
            g.all_reduce(xs, outs=ys, algo=spec)
    torch.cuda.synchronize()
    g.check()
    g.close()


if __name__ == "__main__":
    if sys.argv[1] == "--predict":
        print(json.dumps(predict(sys.argv[2], sys.argv[3])))
    else:
        run(sys.argv[1], sys.argv[2])
