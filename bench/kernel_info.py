#!/usr/bin/env python3
"""VGPRs and resident 512-thread workgroups per CU of every executor / LL / reduce instantiation the runtime
launches (hipFuncGetAttributes + hipOccupancyMaxActiveBlocksPerMultiprocessor), plus a grid sweep of a flat
64 MiB fp32 allreduce with 2 ranks in one launch on one GPU. JSON lines."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.parallel import LocalGroup

    torch.cuda.set_device(0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    protos = {0: "fence", 1: "nts", 2: "wt"}
    for dt in ("float32", "bfloat16", "float16", "fp8_e4m3", "float64", "int32", "int8"):
        for kind, name in ((0, "exec"), (1, "ll"), (2, "reduce")):
            for p in ((0, 1, 2) if kind == 0 else (0,)):
                try:
                    k = nv.kernel_info(dt, "sum", kind, p)
                except nv.FlexarError:
                    continue
                print(json.dumps({"kernel": name, "dtype": dt, "proto": protos[p] if kind == 0 else None, **k,
                                  "resident_blocks": k["blocks_per_cu"] * cus}), flush=True)
    for dt, kind, name in (("bfloat16", 3, "exec_mx fp32 partials"), ("fp8_e4m3", 3, "exec_mx fp32 partials"),
                           ("float32", 4, "exec_mx e4m3 wire"), ("bfloat16", 4, "exec_mx e4m3 wire"),
                           ("float32", 6, "exec_mx MX e4m3 wire"), ("bfloat16", 6, "exec_mx MX e4m3 wire")):
        for p in (0, 2):
            k = nv.kernel_info(dt, "sum", kind, p)
            print(json.dumps({"kernel": name, "dtype": dt, "proto": protos[p], **k,
                              "resident_blocks": k["blocks_per_cu"] * cus}), flush=True)
    # grid sweep: 2 ranks x grid workgroups co-resident in one launch (<= 256 = one per CU)
    grp = LocalGroup(2, workspace_bytes=320 << 20)
    n = (64 << 20) // 4
    xs = [torch.randn(n, device="cuda") for _ in range(2)]
    ys = [torch.empty_like(x) for x in xs]
    for spec in ("flat+pull", "flat+push", "ring"):
        for g in (8, 16, 32, 64, 128):
            grp.set_grid(g)
            for _ in range(3):
                grp.all_reduce(xs, outs=ys, algo=spec)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                grp.all_reduce(xs, outs=ys, algo=spec)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / 10 * 1e3
            print(json.dumps({"sweep": spec, "ranks": 2, "MiB": 64, "grid_per_rank": g, "us": round(us, 1)}),
                  flush=True)
    grp.close()


if __name__ == "__main__":
    main()
