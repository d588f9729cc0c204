#!/usr/bin/env python3
"""Zero-copy flat allreduce ("+zc": peers read the caller's registered IN / OUT, no staging) against the
staging flat schedules, N ranks in one launch on one GPU (LocalGroup: every rank's buffers are plain
device pointers, so no registration is needed). One JSON line per (ranks, spec): kernel time per call,
busbw and the HBM bytes per rank the schedule moves (model: staging flat pull = 2(N-1)/N S + (N+2)/N S +
2(N-1)/N S; zero copy = (N+1)/N S + 2(N-1)/N S; push 2 S; put 2 S + 2(N-1)/N S through the owners'
staging), so the time ratio can be read against the byte ratio.

    python bench/zc_bench.py                      # N = 2, 4, 8 at 64 MiB fp32 per rank
    ZCB_MIB=256 ZCB_RANKS=2 python bench/zc_bench.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    mib = int(os.environ.get("ZCB_MIB", "64"))
    ranks = [int(v) for v in os.environ.get("ZCB_RANKS", "2,4,8").split(",")]
    specs = os.environ.get("ZCB_SPECS", "flat+pull,flat+pull+nts,flat+push,flat+bidir,flat+bidir+wt,flat+zc,flat+zc+nts,flat+zc+wt,flat+zc+push,flat+zc+push+wt,"
                           "flat+zc+put,flat+zc+put+nts").split(",")
    count = (mib << 20) // 4
    for n in ranks:
        grp = LocalGroup(n, workspace_bytes=(4 * mib + 64) << 20)
        xs = [torch.randn(count, device="cuda") for _ in range(n)]
        ys = [torch.empty_like(x) for x in xs]
        ref = torch.stack([x.double() for x in xs]).sum(0)
        for spec in specs:
            for _ in range(2):
                grp.all_reduce(xs, outs=ys, algo=spec)
            torch.cuda.synchronize()
            err = max((y.double() - ref).abs().max().item() for y in ys)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            iters = 10
            a.record()
            for _ in range(iters):
                grp.all_reduce(xs, outs=ys, algo=spec)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / iters
            S = count * 4
            hbm = (S * (1 + 1) if "zc+push" in spec else S * (2 + 2 * (n - 1) / n) if "zc+put" in spec
                   else S * (2 + 4 * (n - 1) / n) if "bidir" in spec
                   else S * ((n + 1) / n + 2 * (n - 1) / n) if "zc" in spec
                   else S * (2 * (n - 1) / n + (n + 2) / n + 2 * (n - 1) / n))
            print(json.dumps({"ranks": n, "MiB_fp32": mib, "spec": spec, "ms": round(ms, 4),
                              "busbw_GBps": round(S / (ms * 1e-3) * 2 * (n - 1) / n / 1e9, 1),
                              "hbm_bytes_per_rank_model": int(hbm),
                              "hbm_TBps_all_ranks": round(n * hbm / (ms * 1e-3) / 1e12, 2),
                              "max_abs_err": err}), flush=True)
        grp.close()
        del xs, ys
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
