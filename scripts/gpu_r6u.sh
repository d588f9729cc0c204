#!/bin/bash
# A/B: fp8 / MX wire transfers instantiated for at most 2 destinations (shipped, FLEXAR_MX_ND2=1) against the
# general one only (abv/mxnd0). HBM bytes (PMC) at 8 ranks, where the fan-in-8 kernel spilled to scratch,
# and time at 8 and 4 ranks, builds alternated.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6u
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
for lib in nd2 nd0; do
  if [ $lib = nd0 ]; then export FLEXAR_LIB_PATH="$R/abv/mxnd0/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && PMC_RANKS=8 PMC_MIB=64 timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv \
        -d "$R/gpurun_out/r6u/pmc_${lib}_$ctr" -o run -- python3 "$R/bench/pmc_model_check.py" flat+pull+mxe4m3 float32 \
        > "$R/gpurun_out/r6u/pmc_${lib}_$ctr.log" 2>&1) || { echo "pmc $lib $ctr failed"; exit 1; }
  done
done
for rep in 1 2 3; do
  for lib in nd2 nd0; do
    if [ $lib = nd0 ]; then export FLEXAR_LIB_PATH="$R/abv/mxnd0/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
    for sd in "flat+pull+mxe4m3@float32@8@64" "flat+pull+mxe4m3@bfloat16@8@64" "flat+pull+mxe5m2@float32@8@64" \
              "flat+pull+mxe4m3@float32@4@100" "flat+pull+mxe4m3@bfloat16@4@100" "fp8@float32@8@64" "fp8@bfloat16@8@64" "fp8@bfloat16@4@100"; do
      IFS=@ read -r spec dt nr mib <<< "$sd"
      line=$(TEP_RANKS=$nr TEP_MIB=$mib timeout -k 10 120 python3 bench/typed_exec_probe.py "$spec" "$dt" \
             2>>gpurun_out/r6u/err.log | grep '^{') || { echo "probe $lib $spec failed"; exit 1; }
      echo "{\"lib\": \"$lib\", \"rep\": $rep, ${line:1}" >> gpurun_out/r6u/time.jsonl
    done
  done
done
# the production kernels (one process per rank: exec_mx_kernel), 8 and 4 ranks sharing the GPU
for rep in 1 2; do
  for lib in nd2 nd0; do
    if [ $lib = nd0 ]; then export FLEXAR_LIB_PATH="$R/abv/mxnd0/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
    for nr in 8 4; do
      GPU_MAX_HW_QUEUES=2 TMP_RANKS=$nr TMP_MIB=64 timeout -k 10 300 python3 bench/typed_mp_probe.py flat:float32 mx:float32 \
          mx:bfloat16 fp8:bfloat16 2>>gpurun_out/r6u/err.log | grep '^{' | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" \
          >> gpurun_out/r6u/mp.jsonl || { echo "mp probe $lib $nr failed"; exit 1; }
    done
  done
done
unset FLEXAR_LIB_PATH
python3 - <<'PY' | tee gpurun_out/r6u/summary.txt
import csv, glob, json, os, subprocess, sys
p = json.loads(subprocess.run([sys.executable, "bench/pmc_model_check.py", "--predict", "flat+pull+mxe4m3", "float32"],
                              capture_output=True, text=True, env=dict(os.environ, PMC_RANKS="8", PMC_MIB="64")).stdout)
print("model (8 ranks x 64 MiB):", round(p["read_MiB"], 1), "MiB read,", round(p["write_MiB"], 1), "MiB written")
for f in sorted(glob.glob("gpurun_out/r6u/pmc_*/run_counter_collection.csv")):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "group_kernel" in r["Kernel_Name"]]
    tag = f.split("/")[-2]
    k = 2 if "FETCH" in tag else 1
    print(tag, round(k * sum(vals) / len(vals) / 1024, 1), "MiB per dispatch")
rows = {}
for l in open("gpurun_out/r6u/time.jsonl"):
    d = json.loads(l)
    rows.setdefault((d["spec"], d["dtype"], d["ranks"]), {}).setdefault(d["lib"], []).append(d["us_per_call"])
for k, v in rows.items():
    print(k, {lib: sorted(x) for lib, x in v.items()})
mp = {}
for l in open("gpurun_out/r6u/mp.jsonl"):
    d = json.loads(l)
    mp.setdefault((d["case"], d["ranks"]), {}).setdefault(d["lib"], []).append(d["us_per_call"])
print("one process per rank (exec_mx_kernel), 64 MiB per rank:")
for k, v in sorted(mp.items()):
    print(k, {lib: sorted(x) for lib, x in v.items()})
PY
