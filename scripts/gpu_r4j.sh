#!/bin/bash
# Round 4, tenth GPU pass: the MX wire's cost - hipEvent time per call (4 ranks in one launch, 100 MiB per
# rank) for the global-scale fp8 wire (amax pass + executor), the MX wire (executor only) and the untyped
# flat, then a kernel trace of each for per-kernel times. Each GPU step bounded; chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4j
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r4j
: > $O/mx_ab.jsonl
for rep in 1 2; do
  for dt in bfloat16 float32; do
    for spec in fp8 flat+pull+mxe4m3 flat+pull; do
      timeout -k 10 120 python3 bench/typed_exec_probe.py $spec $dt >> $O/mx_ab.jsonl || exit 1
    done
  done
done
cat $O/mx_ab.jsonl
for spec in fp8 flat+pull+mxe4m3; do
  tag=$(echo $spec | tr '+' '_')
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python3 bench/typed_exec_probe.py $spec bfloat16 \
      > $O/prof_$tag.json 2>&1 || exit 1
done
echo profiles ok
