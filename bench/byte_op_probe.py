#!/usr/bin/env python3
"""8-bit PROD / MAX / MIN allreduces in one launch (LocalGroup), hipEvent-timed: the A/B of FLEXAR_BYTE_OP_U1
(one 16-B group per lane for 8-bit byte arithmetic). JSON lines: spec, dtype, op, us per call, exact."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    n = int(os.environ.get("BOP_RANKS", "4"))
    mib = int(os.environ.get("BOP_MIB", "64"))
    iters = int(os.environ.get("BOP_ITERS", "10"))
    grp = LocalGroup(n, workspace_bytes=6 * (mib << 20) + (64 << 20))
    lib = os.path.basename(os.path.dirname(os.environ.get("FLEXAR_LIB_PATH", "") or "_lib/x"))
    for dt in (torch.int8, torch.uint8):
        count = mib << 20
        g = torch.Generator(device="cuda").manual_seed(7)
        xs = [torch.randint(0, 4, (count,), device="cuda", generator=g, dtype=torch.int32).to(dt) for _ in range(n)]
        for op in ("max", "min", "prod"):
            ref = xs[0].to(torch.int64)
            for x in xs[1:]:
                ref = torch.maximum(ref, x.to(torch.int64)) if op == "max" else \
                    torch.minimum(ref, x.to(torch.int64)) if op == "min" else ref * x.to(torch.int64)
            ref = ref.to(dt)
            for spec in ("flat+pull", "flat+pull+wt", "ring"):
                ys = [torch.empty_like(x) for x in xs]
                run = lambda: grp.all_reduce(xs, op, outs=ys, algo=spec)  # noqa: E731
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(iters):
                    run()
                b.record()
                torch.cuda.synchronize()
                exact = all(bool(torch.equal(y, ref)) for y in ys)
                print(json.dumps({"lib": lib, "spec": spec, "dtype": str(dt).split(".")[-1], "op": op,
                                  "us_per_call": round(a.elapsed_time(b) * 1e3 / iters, 1), "exact": exact}), flush=True)
    grp.check()
    grp.close()


if __name__ == "__main__":
    main()
