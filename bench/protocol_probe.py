#!/usr/bin/env python3
"""Per-kernel protocol cost on one GPU (run under rocprofv3 --kernel-trace): LocalGroup allreduce of
tiny/medium buffers with each algorithm and workgroup count, so kernel durations isolate launch-free
protocol costs (SIGNAL release + WAIT acquire per stage, LL granules, per-workgroup latency chains).

Writes a manifest (one entry per launch group, in launch order) so `--parse` can align the
rocprofv3 kernel trace with (ranks, size, spec, grid):

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 bench/protocol_probe.py --manifest M
    python3 bench/protocol_probe.py --parse OUT/run_kernel_trace.csv --manifest M
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(args):
    import torch

    from allreduce_over_mpi_amd.parallel import LocalGroup

    dev = torch.device("cuda", 0)
    manifest = []
    for nr in [int(v) for v in args.ranks.split(",")]:
        kibs = [int(v) for v in args.kib.split(",")]
        g = LocalGroup(nr, workspace_bytes=max(128 << 20, 4 * nr * max(kibs) << 10))  # one piece per call
        for kib in [int(v) for v in args.kib.split(",")]:
            n = kib * 256
            xs = [torch.randn(n, device=dev) for _ in range(nr)]
            ys = [torch.empty_like(x) for x in xs]
            for spec in args.specs.split(","):
                for grid in [int(v) for v in args.grids.split(",")]:
                    if grid * nr > 256 or (spec == "ll" and (kib > 1024 or grid != 1)):
                        continue  # LL picks its own grid
                    g.set_grid(grid)
                    for _ in range(args.reps):
                        g.all_reduce(xs, outs=ys, algo=spec)
                    manifest.append({"ranks": nr, "kib": kib, "spec": spec, "grid": grid, "reps": args.reps})
        torch.cuda.synchronize()
        g.close()
    with open(args.manifest, "w") as f:
        json.dump(manifest, f)


def parse(args):
    import csv

    rows = [r for r in csv.DictReader(open(args.parse)) if "flexar" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    man = json.load(open(args.manifest))
    assert sum(m["reps"] for m in man) == len(rows), (sum(m["reps"] for m in man), len(rows))
    i = 0
    out = []
    for m in man:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[i:i + m["reps"]]]
        i += m["reps"]
        out.append(dict(m, kernel=rows[i - 1]["Kernel_Name"].split("(")[0][-40:], median_us=round(statistics.median(d), 2)))
    for o in out:
        print(json.dumps(o))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,8")
    ap.add_argument("--kib", default="4,64,256,1024,4096")
    ap.add_argument("--specs", default="ll,oneshot,flat+pull,flat+push,ring")
    ap.add_argument("--grids", default="1,2,4,8,16,32")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--manifest", default="gpurun_out/probe_manifest.json")
    ap.add_argument("--parse", default="")
    args = ap.parse_args()
    parse(args) if args.parse else run(args)


if __name__ == "__main__":
    main()
