#!/bin/bash
# Program-cost model vs measured HBM bytes: one rocprofv3 pass per (spec, counter) - FETCH_SIZE and
# WRITE_SIZE cannot share a pass (3 + 2 TCC counters > 4) - 4 ranks in one launch, 64 MiB per rank.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/pmc_model
export FLEXAR_NO_BUILD=1
SPECS="${PMC_SPECS:-flat+pull@float32 flat+push@float32 ring@float32 rhd+pull@float32 tree:2,2+push@float32 oneshot@float32 \
flat+zc+push@float32 ring+f32@bfloat16 ring+rw@bfloat16 rhd+pull+f32@bfloat16 rhd+pull+rw@bfloat16 fp8@float32 fp8@bfloat16}"
run() {  # spec dtype counter
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc "$3" --output-format csv \
      -d "$R/gpurun_out/pmc_model/$1_$2_$3" -o run -- python3 "$R/bench/pmc_model_check.py" "$1" "$2" \
      > "$R/gpurun_out/pmc_model/$1_$2_$3.log" 2>&1)
}
rc=0
for sd in $SPECS; do
  spec=${sd%@*}; dt=${sd##*@}
  run "$spec" "$dt" FETCH_SIZE && run "$spec" "$dt" WRITE_SIZE || { rc=$?; break; }
done
python3 - <<'PY' > gpurun_out/pmc_model/summary.txt
import csv, glob, json, subprocess, sys
rows = {}
for f in sorted(glob.glob("gpurun_out/pmc_model/*/run_counter_collection.csv")):
    tag = f.split("/")[-2]
    spec, dt, c1, c2 = tag.rsplit("_", 3)  # "<spec>_<dtype>_FETCH_SIZE"
    ctr = c1 + "_" + c2
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if "exec_group_kernel" in r["Kernel_Name"] or "exec_mx_group_kernel" in r["Kernel_Name"]]
    if vals:
        rows.setdefault((spec, dt), {})[ctr] = sum(vals) / len(vals) / 1024  # KiB -> MiB per dispatch
print(f"{'spec':18s} {'dtype':9s} {'model read':>11s} {'FETCH':>9s} {'FETCHx2':>9s} {'model write':>12s} {'WRITE':>9s}  (MiB per dispatch, 4 ranks x 64 MiB)")
for (spec, dt), v in sorted(rows.items()):
    p = json.loads(subprocess.run([sys.executable, "bench/pmc_model_check.py", "--predict", spec, dt],
                                  capture_output=True, text=True).stdout)
    f2 = 2 * v.get("FETCH_SIZE", float("nan"))
    w = v.get("WRITE_SIZE", float("nan"))
    print(f"{spec:18s} {dt:9s} {p['read_MiB']:11.1f} {f2 / 2:9.1f} {f2:9.1f} {p['write_MiB']:12.1f} {w:9.1f}   "
          f"read {f2 / p['read_MiB']:.3f}x  write {w / p['write_MiB']:.3f}x")
PY
cat gpurun_out/pmc_model/summary.txt
exit $rc
