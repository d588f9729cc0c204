#!/bin/bash
# Round 6 A/B: channel -> workgroup mapping. Shipped: channel c = workgroups b == c (mod C). Variant (abv/,
# FLEXAR_CHAN_CONTIG=1): contiguous workgroups per channel. HBM counters (FETCH_SIZE) and time, 4 / 8 ranks in one
# launch on one GPU. Each step bounded.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6l
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
for lib in base contig; do
  if [ $lib = contig ]; then export FLEXAR_LIB_PATH="$R/abv/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
  for spec in "tree:4+pull" "tree:4:3+pull" "tree:2,2:3+pull"; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/r6l/pmc_${lib}_$spec" \
        -o run -- python3 "$R/bench/pmc_model_check.py" "$spec" float32 > "$R/gpurun_out/r6l/pmc_${lib}_$spec.log" 2>&1) ||
        { echo "pmc $lib $spec failed"; exit 1; }
  done
  for rep in 1 2; do
    for spec in "flat+pull" "rhd+pull" "tree:2,2,2:7+pull" "tree:4,2:7+pull"; do
      line=$(TEP_GRID=28 TEP_RANKS=8 TEP_MIB=64 timeout -k 10 120 python3 bench/typed_exec_probe.py "$spec" float32 \
             2>>gpurun_out/r6l/err.log | grep '^{') || { echo "probe $lib $spec failed"; exit 1; }
      echo "{\"lib\": \"$lib\", \"rep\": $rep, ${line:1}" >> gpurun_out/r6l/time.jsonl
    done
  done
done
unset FLEXAR_LIB_PATH
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob("gpurun_out/r6l/pmc_*/run_counter_collection.csv")):
    tag = f.split("/")[-2]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "exec_group_kernel" in r["Kernel_Name"]]
    print(tag, round(2 * sum(vals) / len(vals) / 1024, 1), "MiB read per dispatch")
PY
cat gpurun_out/r6l/time.jsonl
