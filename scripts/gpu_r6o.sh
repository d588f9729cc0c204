#!/bin/bash
# Follow-up of gpu_r6n.sh: are the channelled flat schedule's extra L2 requests reads or writes, hits or misses,
# and do the CUs issue them (TCP -> TCC requests)? 4 ranks x 64 MiB fp32 in one launch.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6o
export FLEXAR_NO_BUILD=1
run() {  # spec counters tag
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv \
      -d "$R/gpurun_out/r6o/$1_$3" -o run -- python3 "$R/bench/pmc_model_check.py" "$1" float32 \
      > "$R/gpurun_out/r6o/$1_$3.log" 2>&1)
}
for spec in flat+pull tree:4:3+pull; do
  run "$spec" "TCC_READ_sum TCC_WRITE_sum TCC_HIT_sum TCC_MISS_sum" tcc || exit $?
  run "$spec" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum" tcp || exit $?
  run "$spec" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU" sq || exit $?
done
python3 - <<'PY' | tee gpurun_out/r6o/summary.txt
import csv, glob
for f in sorted(glob.glob("gpurun_out/r6o/*/run_counter_collection.csv")):
    tag = f.split("/")[-2]
    acc = {}
    for r in csv.DictReader(open(f)):
        if "exec_group_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(tag, {k: round(sum(v) / len(v), 1) for k, v in acc.items()})
PY
