#!/usr/bin/env python3
"""Per-kernel device time from rocprofv3 --kernel-trace --stats runs laid out DIR/<lib>/<case>.<rep>/...: the
rocpd SQLite database (`*_results.db`, rocprofv3's default output on ROCm 7.2; its `top_kernels` view) or a
`*kernel_stats.csv` (--output-format csv). One line per (lib, case): the average time of the executor kernels
(exec_*) and of the amax pass in us, averaged over the repetitions.

    python3 bench/kstats_summary.py DIR            # A/B table
    python3 bench/kstats_summary.py --top FILE.db  # the top kernels of one run as CSV (name,calls,total_us,avg_us,pct)
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def top_kernels(path):
    """[(name, calls, total_us, avg_us, pct)] of one run (db or csv)."""
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
        con.close()
        return [(n, int(c), float(t), float(a), float(p)) for n, c, t, a, p in rows]
    out = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["Percentage"])))
    return out


def main(root):
    rows = defaultdict(list)
    files = glob.glob(os.path.join(root, "*", "*", "**", "*_results.db"), recursive=True) + \
        glob.glob(os.path.join(root, "*", "*", "**", "*kernel_stats.csv"), recursive=True)
    for f in files:
        rel = os.path.relpath(f, root).split(os.sep)
        lib, case = rel[0], rel[1].rsplit(".", 1)[0]
        per = defaultdict(float)
        for name, calls, _, avg, _ in top_kernels(f):
            key = "exec" if "exec" in name else ("amax" if "amax" in name else None)
            if key and calls >= 10:
                per[key] += avg
        rows[(lib, case)].append(per)
    for (lib, case), pers in sorted(rows.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        ex = sum(p["exec"] for p in pers) / len(pers)
        am = sum(p["amax"] for p in pers) / len(pers)
        print(f"{case:32s} {lib:5s} exec {ex:8.1f} us  amax {am:6.1f} us  ({len(pers)} runs)")


if __name__ == "__main__":
    if sys.argv[1] == "--top":
        w = csv.writer(sys.stdout)
        w.writerow(["name", "calls", "total_us", "avg_us", "pct"])
        for r in top_kernels(sys.argv[2]):
            w.writerow([r[0][:160], r[1], round(r[2], 3), round(r[3], 3), round(r[4], 2)])
    else:
        main(sys.argv[1])
