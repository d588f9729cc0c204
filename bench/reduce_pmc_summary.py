#!/usr/bin/env python3
"""Counter summary of the standalone reduction (scripts/gpu_r5o.sh): per (dtype, fan-in), the reduce_kernel
dispatches' mean FETCH_SIZE / WRITE_SIZE against the bytes the kernel must move (K sources read, one destination
written), the SQ wave-cycle split and LDS activity, and the rate those bytes give over the kernel-trace time.

    python3 bench/reduce_pmc_summary.py gpurun_out/r5o
"""
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def counters(d):
    tot = defaultdict(float)
    disp = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "reduce_kernel" not in r.get("Kernel_Name", ""):
                continue
            disp.add(r.get("Dispatch_Id", ""))
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    n = max(1, len(disp))
    return {k: v / n for k, v in tot.items()}, len(disp)


def trace_times(root):
    """reduce_kernel durations (us) in dispatch order, from the kernel-trace database."""
    dbs = glob.glob(os.path.join(root, "trace", "**", "*.db"), recursive=True)
    if not dbs:
        return []
    con = sqlite3.connect(dbs[0])
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    return [(n, (e - s) / 1e3) for n, s, e in rows if "reduce_kernel" in n]


def main(root):
    es = {"float32": 4, "bfloat16": 2, "float8_e4m3fn": 1}
    nbytes = 256 << 20
    out = []
    for dt in ("float32", "bfloat16", "float8_e4m3fn"):
        for k in (2, 8):
            f, nf = counters(os.path.join(root, f"{dt}_k{k}_FETCH_SIZE"))
            w, _ = counters(os.path.join(root, f"{dt}_k{k}_WRITE_SIZE"))
            s, _ = counters(os.path.join(root, f"{dt}_k{k}_SQ"))
            if not nf:
                continue
            read_need, write_need = k * nbytes, nbytes
            row = {"dtype": dt, "fanin": k, "dispatches": nf,
                   "FETCH_SIZE_KiB": round(f.get("FETCH_SIZE", 0)), "WRITE_SIZE_KiB": round(w.get("WRITE_SIZE", 0)),
                   "read_need_KiB": read_need // 1024, "write_need_KiB": write_need // 1024}
            row["fetch_over_need"] = round(f.get("FETCH_SIZE", 0) * 1024 / read_need, 3)
            row["write_over_need"] = round(w.get("WRITE_SIZE", 0) * 1024 / write_need, 3)
            cyc = s.get("SQ_WAVE_CYCLES", 0) or 1
            row["wait_any_pct"] = round(100 * s.get("SQ_WAIT_ANY", 0) / cyc, 1)
            row["valu_active_pct"] = round(100 * s.get("SQ_ACTIVE_INST_VALU", 0) / cyc, 1)
            row["lds_insts"] = s.get("SQ_INSTS_LDS", 0)
            row["lds_bank_conflict_cycles"] = s.get("SQ_LDS_BANK_CONFLICT", 0)
            out.append(row)
    times = trace_times(root)
    # per dtype (by kernel name), kernel_bench's order: fan-in 2 then 8, each case 3 warm-up + 5 timed calls
    token = {"float32": "reduce_kernel<float", "bfloat16": "bf16_t", "float8_e4m3fn": "fp8e4m3_t"}
    per = 8
    seen = defaultdict(int)
    for row in out:
        mine = [t for n, t in times if token[row["dtype"]] in n]
        i = seen[row["dtype"]]
        seen[row["dtype"]] += per
        ts = mine[i:i + per]
        if ts:
            us = sorted(ts)[len(ts) // 2]
            row["kernel_us_median"] = round(us, 1)
            moved = row["FETCH_SIZE_KiB"] * 1024 + row["WRITE_SIZE_KiB"] * 1024
            row["counter_TBps"] = round(moved / (us * 1e-6) / 1e12, 3)
            row["model_TBps"] = round((row["fanin"] + 1) * nbytes / (us * 1e-6) / 1e12, 3)
    for row in out:
        print(json.dumps(row))


if __name__ == "__main__":
    main(sys.argv[1])
