#!/bin/bash
# Final tree: rocprofv3 kernel trace + stats of the N = 1 bench (reduce_kernel and group_executor sections included).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6_prof
export FLEXAR_NO_BUILD=1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/r6_prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/r6_prof/bench.log" 2>&1)
rc=$?
f=$(ls gpurun_out/r6_prof/*kernel_stats.csv gpurun_out/r6_prof/*/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY' | tee gpurun_out/r6_prof/top_kernels.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"{'kernel':90s} {'calls':>6s} {'total ms':>9s} {'avg us':>9s}")
for r in rows[:25]:
    print(f"{r['Name'][:90]:90s} {int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e6:9.2f} {float(r['AverageNs'])/1e3:9.1f}")
PY
exit $rc
