#!/bin/bash
# Counter audit of the executors after the slice change: HBM fetch / write and L1 -> L2 line requests per dispatch
# against the program-cost model, 8 ranks x 64 MiB in one launch (the 8-GPU node's schedules), untyped and typed.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6r
export FLEXAR_NO_BUILD=1 PMC_RANKS=8 PMC_MIB=64
run() {  # spec dtype counters tag
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $3 --output-format csv \
      -d "$R/gpurun_out/r6r/$1_$2_$4" -o run -- python3 "$R/bench/pmc_model_check.py" "$1" "$2" \
      > "$R/gpurun_out/r6r/$1_$2_$4.log" 2>&1)
}
for sd in flat+pull@float32 flat+push@float32 flat+zc+push@float32 rhd:7+pull@float32 tree:4,2:7+pull@float32 \
          ring:7@float32 flat+pull+f32@bfloat16 fp8@bfloat16 flat+pull+mxe4m3@float32; do
  spec=${sd%@*}; dt=${sd##*@}
  run "$spec" "$dt" FETCH_SIZE fetch && run "$spec" "$dt" WRITE_SIZE write &&
  run "$spec" "$dt" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" tcp || exit $?
done
python3 - <<'PY' | tee gpurun_out/r6r/summary.txt
import csv, glob, json, subprocess, sys
rows = {}
for f in sorted(glob.glob("gpurun_out/r6r/*/run_counter_collection.csv")):
    spec, dt, _ = f.split("/")[-2].rsplit("_", 2)
    for r in csv.DictReader(open(f)):
        if "group_kernel" in r["Kernel_Name"]:
            rows.setdefault((spec, dt), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
print(f"{'spec':22s} {'dtype':9s} {'model rd':>9s} {'2xFETCH':>9s} {'model wr':>9s} {'WRITE':>9s} {'L1rd MiB':>9s} {'L1wr MiB':>9s}")
for (spec, dt), v in sorted(rows.items()):
    m = {k: sum(x) / len(x) for k, x in v.items()}
    p = json.loads(subprocess.run([sys.executable, "bench/pmc_model_check.py", "--predict", spec, dt],
                                  capture_output=True, text=True).stdout)
    f2 = 2 * m.get("FETCH_SIZE", float("nan")) / 1024
    w = m.get("WRITE_SIZE", float("nan")) / 1024
    l1r = m.get("TCP_TCC_READ_REQ_sum", float("nan")) * 128 / 2**20
    l1w = m.get("TCP_TCC_WRITE_REQ_sum", float("nan")) * 64 / 2**20
    print(f"{spec:22s} {dt:9s} {p['read_MiB']:9.1f} {f2:9.1f} {p['write_MiB']:9.1f} {w:9.1f} {l1r:9.1f} {l1w:9.1f}"
          f"   rd {f2 / p['read_MiB']:.3f}x wr {w / p['write_MiB']:.3f}x")
PY
