#!/bin/bash
# Round 6 A/B: slice boundaries in 256-B runs (shipped, FLEXAR_SLICE_ALIGN=256) against 16 B (abv/slice16). L2 requests
# and HBM fetch (rocprofv3 PMC) and time (LocalGroup, one launch) for untyped, typed and channelled schedules.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6p
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
for lib in a256 a16; do
  if [ $lib = a16 ]; then export FLEXAR_LIB_PATH="$R/abv/slice16/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
  for spec in "flat+pull" "tree:4:3+pull" "rhd+pull"; do
    for ctr in "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
      tag="${lib}_${spec}_${ctr%% *}"
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/r6p/pmc_$tag" \
          -o run -- python3 "$R/bench/pmc_model_check.py" "$spec" float32 > "$R/gpurun_out/r6p/pmc_$tag.log" 2>&1) ||
          { echo "pmc $tag failed"; exit 1; }
    done
  done
  for rep in 1 2; do
    for sd in "flat+pull@float32@4@100@" "flat+push@float32@4@100@" "ring@float32@4@100@" "rhd+pull@float32@4@100@" \
              "tree:4:3+pull@float32@4@100@" "fp8@bfloat16@4@100@" "flat+pull+f32@bfloat16@4@100@" \
              "flat+pull+mxe4m3@float32@4@100@" "flat+pull@float32@8@64@28" "tree:2,2,2:7+pull@float32@8@64@28" \
              "tree:4,2:7+pull@float32@8@64@28"; do
      IFS=@ read -r spec dt nr mib grid <<< "$sd"
      line=$(TEP_GRID=$grid TEP_RANKS=$nr TEP_MIB=$mib timeout -k 10 120 python3 bench/typed_exec_probe.py "$spec" "$dt" \
             2>>gpurun_out/r6p/err.log | grep '^{') || { echo "probe $lib $spec failed"; exit 1; }
      echo "{\"lib\": \"$lib\", \"rep\": $rep, ${line:1}" >> gpurun_out/r6p/time.jsonl
    done
  done
done
unset FLEXAR_LIB_PATH
python3 - <<'PY' | tee gpurun_out/r6p/summary.txt
import csv, glob, json
for f in sorted(glob.glob("gpurun_out/r6p/pmc_*/run_counter_collection.csv")):
    tag = f.split("/")[-2]
    acc = {}
    for r in csv.DictReader(open(f)):
        if "exec_group_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(tag, {k: round(sum(v) / len(v), 1) for k, v in acc.items()})
rows = {}
for l in open("gpurun_out/r6p/time.jsonl"):
    d = json.loads(l)
    rows.setdefault((d["spec"], d["dtype"], d["ranks"]), {}).setdefault(d["lib"], []).append(d["us_per_call"])
for k, v in rows.items():
    print(k, {lib: sorted(x) for lib, x in v.items()})
PY
