#!/bin/bash
# Typed executors vs the untyped one: effective HBM rate (model bytes / hipEvent time) and per-kernel time
# (rocprofv3 --kernel-trace --stats), 4 ranks in one launch, 100 MiB per rank. One process per case.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/typed_probe
export FLEXAR_NO_BUILD=1
rc=0
for c in "flat+pull float32" "fp8 float32" "fp8 bfloat16" "flat+pull bfloat16" "rhd+pull+rw bfloat16" "rhd+pull+f32 bfloat16" \
         "ring+rw bfloat16" "ring+f32 bfloat16"; do
  set -- $c
  tag="$1_$2"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/typed_probe/$tag" -o run -- python3 "$R/bench/typed_exec_probe.py" "$1" "$2" \
      > "$R/gpurun_out/typed_probe/$tag.log" 2>&1) || { rc=$?; break; }
  grep '^{' "gpurun_out/typed_probe/$tag.log" >> gpurun_out/typed_probe/summary.jsonl
  grep -h "exec\|amax" "gpurun_out/typed_probe/$tag/run_kernel_stats.csv" | cut -d, -f1-4 | sed "s/^/$tag /" >> gpurun_out/typed_probe/kernels.txt
done
cat gpurun_out/typed_probe/summary.jsonl; cat gpurun_out/typed_probe/kernels.txt | cut -c1-220
exit $rc
