#!/bin/bash
# Typed-executor ratios after the scratch-free change (the VERDICT r5 targets: fp8 wire / bf16 input <= 0.75x and
# MX wire / fp32 input <= 0.70x of the untyped flat on the same input), 4 ranks x 100 MiB: one process per rank
# (production kernels) and one launch (LocalGroup), 3 repetitions.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6w
export FLEXAR_NO_BUILD=1
for rep in 1 2 3; do
  TMP_RANKS=4 TMP_MIB=100 timeout -k 10 300 python3 bench/typed_mp_probe.py flat:float32 flat:bfloat16 fp8:bfloat16 \
      mx:float32 mx:bfloat16 2>>gpurun_out/r6w/err.log | grep '^{' >> gpurun_out/r6w/mp.jsonl || { echo "mp failed"; exit 1; }
  for sd in "flat+pull@float32" "flat+pull@bfloat16" "fp8@bfloat16" "flat+pull+mxe4m3@float32" "flat+pull+mxe4m3@bfloat16"; do
    spec=${sd%@*}; dt=${sd##*@}
    TEP_RANKS=4 TEP_MIB=100 timeout -k 10 120 python3 bench/typed_exec_probe.py "$spec" "$dt" 2>>gpurun_out/r6w/err.log \
        | grep '^{' >> gpurun_out/r6w/group.jsonl || { echo "group $spec failed"; exit 1; }
  done
done
python3 - <<'PY' | tee gpurun_out/r6w/summary.txt
import json, statistics as st
mp, gr = {}, {}
for l in open("gpurun_out/r6w/mp.jsonl"):
    d = json.loads(l); mp.setdefault(d["case"], []).append(d["us_per_call"])
for l in open("gpurun_out/r6w/group.jsonl"):
    d = json.loads(l); gr.setdefault((d["spec"], d["dtype"]), []).append(d["us_per_call"])
m = {k: st.median(v) for k, v in mp.items()}
g = {k: st.median(v) for k, v in gr.items()}
print("one process per rank (median us):", m)
print("  fp8 wire / bf16 flat:", round(m["fp8:bfloat16"] / m["flat:bfloat16"], 3), " MX / fp32 flat:",
      round(m["mx:float32"] / m["flat:float32"], 3), " MX bf16 / bf16 flat:", round(m["mx:bfloat16"] / m["flat:bfloat16"], 3))
print("one launch (median us):", g)
print("  fp8 wire / bf16 flat:", round(g[("fp8", "bfloat16")] / g[("flat+pull", "bfloat16")], 3), " MX / fp32 flat:",
      round(g[("flat+pull+mxe4m3", "float32")] / g[("flat+pull", "float32")], 3), " MX bf16 / bf16 flat:",
      round(g[("flat+pull+mxe4m3", "bfloat16")] / g[("flat+pull", "bfloat16")], 3))
PY
