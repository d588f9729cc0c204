#!/bin/bash
# Follow-up of gpu_r6p.sh: the two cases where 256-B slice boundaries measured slower (rhd:7 at 8 ranks, bf16 with
# fp32 partials), 4 repetitions alternating the two builds so box drift hits both alike.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6q
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
for rep in 1 2 3 4; do
  for lib in a256 a16; do
    if [ $lib = a16 ]; then export FLEXAR_LIB_PATH="$R/abv/slice16/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
    for sd in "flat+pull+f32@bfloat16@4@100@" "rhd+pull+f32@bfloat16@4@100@" "tree:2,2,2:7+pull@float32@8@64@28" \
              "tree:2,2,2:7+pull@float32@8@64@" "rhd+pull@float32@8@64@28" "tree:4:3+pull@float32@4@100@"; do
      IFS=@ read -r spec dt nr mib grid <<< "$sd"
      line=$(TEP_GRID=$grid TEP_RANKS=$nr TEP_MIB=$mib timeout -k 10 120 python3 bench/typed_exec_probe.py "$spec" "$dt" \
             2>>gpurun_out/r6q/err.log | grep '^{') || { echo "probe $lib $spec failed"; exit 1; }
      echo "{\"lib\": \"$lib\", \"rep\": $rep, \"grid\": \"$grid\", ${line:1}" >> gpurun_out/r6q/time.jsonl
    done
  done
done
python3 - <<'PY' | tee gpurun_out/r6q/summary.txt
import json
rows = {}
for l in open("gpurun_out/r6q/time.jsonl"):
    d = json.loads(l)
    rows.setdefault((d["spec"], d["dtype"], d["ranks"], d["grid"]), {}).setdefault(d["lib"], []).append(d["us_per_call"])
for k, v in rows.items():
    print(k, {lib: sorted(x) for lib, x in v.items()})
PY
