#!/bin/bash
# Where do the channelled programs' extra ~3 % HBM fetches come from? Hypothesis: the WAIT polls (8-byte
# system-scope loads of uncached flags) count as 32-byte EA read requests. Split FETCH into 32 B / all
# requests for the flat schedule unsplit and split into 3 channels (4 ranks x 64 MiB, one launch).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6n
export FLEXAR_NO_BUILD=1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --list-avail > "$R/gpurun_out/r6n/avail.txt" 2>&1) || exit $?
grep -oE "TCC_EA0?_RD[A-Z0-9_]*|TCC_UC[A-Z0-9_]*|TCC_NC[A-Z0-9_]*|TCC_REQ[A-Z0-9_]*|TCC_READ[A-Z0-9_]*" gpurun_out/r6n/avail.txt | sort -u > gpurun_out/r6n/tcc_names.txt || true
cat gpurun_out/r6n/tcc_names.txt
run() {  # spec counters tag
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv \
      -d "$R/gpurun_out/r6n/$1_$3" -o run -- python3 "$R/bench/pmc_model_check.py" "$1" float32 \
      > "$R/gpurun_out/r6n/$1_$3.log" 2>&1)
}
for spec in flat+pull tree:4:3+pull; do
  run "$spec" "FETCH_SIZE" fetch || exit $?
  run "$spec" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum" rdreq || exit $?
  run "$spec" "TCC_UC_REQ_sum TCC_REQ_sum" ucreq || exit $?
done
python3 - <<'PY' | tee gpurun_out/r6n/summary.txt
import csv, glob
for f in sorted(glob.glob("gpurun_out/r6n/*/run_counter_collection.csv")):
    tag = f.split("/")[-2]
    acc = {}
    for r in csv.DictReader(open(f)):
        if "exec_group_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(tag, {k: round(sum(v) / len(v), 1) for k, v in acc.items()})
PY
