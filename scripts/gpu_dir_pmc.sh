#!/bin/bash
# HBM bytes of the link-direction schedules (flat+bidir, flat+zc+put) next to flat+push and flat+zc+push: rocprofv3 FETCH_SIZE and WRITE_SIZE, one
# counter and one spec per pass (kernels of both specs share a name), N=2 ranks in one launch, 64 MiB fp32.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/dir_pmc
export FLEXAR_NO_BUILD=1
run() {  # spec counter
  (cd /tmp && export TMPDIR=/tmp && ZCB_RANKS=2 ZCB_SPECS="$1" timeout -s KILL 120 rocprofv3 --pmc "$2" --output-format csv \
      -d "$R/gpurun_out/dir_pmc/$1_$2" -o run -- python3 "$R/bench/zc_bench.py" > "$R/gpurun_out/dir_pmc/$1_$2.log" 2>&1)
}
run flat+push FETCH_SIZE && run flat+push WRITE_SIZE && run flat+bidir FETCH_SIZE && run flat+bidir WRITE_SIZE &&
  run flat+zc+push FETCH_SIZE && run flat+zc+push WRITE_SIZE && run flat+zc+put FETCH_SIZE && run flat+zc+put WRITE_SIZE && echo "pmc ok"
rc=$?
python3 - <<'PY' > gpurun_out/dir_pmc/summary.txt
import csv, glob, os
for f in sorted(glob.glob("gpurun_out/dir_pmc/*/run_counter_collection.csv")):
    tag = f.split("/")[-2]
    acc = {}
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "exec_group_kernel" not in k:
            continue
        acc.setdefault(k, [0, 0.0])
        acc[k][0] += 1
        acc[k][1] += float(row["Counter_Value"])
    for k, (n, v) in acc.items():
        print(f"{tag:24s} {k[:60]:60s} dispatches={n:3d} MB/dispatch={v / n / 1024:9.2f}")
PY
cat gpurun_out/dir_pmc/summary.txt
exit $rc
