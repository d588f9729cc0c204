#!/usr/bin/env python3
"""Per-kernel SQ counter summary of rocprofv3 --pmc runs (scripts/gpu_typed_pmc.sh): for every executor kernel,
the wave-cycle split (SQ_WAIT_ANY = parked on s_waitcnt / barriers, SQ_WAIT_INST_ANY = issue stalls,
SQ_ACTIVE_INST_ANY = issuing; together ~ SQ_WAVE_CYCLES), VALU activity and VALU instructions per wave.

    python3 bench/pmc_sq_summary.py gpurun_out/typed_pmc
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "*/"))):
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        tot = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "")
                    if "exec" not in k:
                        continue
                    short = k.split("(")[0].replace("void ", "").replace("flexar::", "")
                    tot[short][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[short].add(row.get("Dispatch_Id", ""))
        for k, c in tot.items():
            wc = c.get("SQ_WAVE_CYCLES", 0) or 1.0
            waves = c.get("SQ_WAVES", 0) or 1.0
            print(f"{os.path.basename(d.rstrip('/')):22s} {k[:60]:60s} dispatches {len(disp[k]):3d} "
                  f"wait_any {c.get('SQ_WAIT_ANY', 0) / wc:6.1%} wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wc:6.1%} "
                  f"active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1%} valu_active {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:6.1%} "
                  f"valu_insts/wave {c.get('SQ_INSTS_VALU', 0) / waves:10.0f} busy_cycles {c.get('SQ_BUSY_CYCLES', 0):.3g}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/typed_pmc")
