#!/bin/bash
# Round 4: the fp8 wires at DDP bucket size (25 MiB fp32 per rank), 2 and 4 ranks in one launch.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4r
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4r
: > $O/bucket.jsonl
for n in 2 4; do
  for spec in fp8 flat+pull+mxe4m3 flat+pull; do
    TEP_RANKS=$n TEP_MIB=25 TEP_ITERS=20 timeout -k 10 120 python3 bench/typed_exec_probe.py $spec float32 >> $O/bucket.jsonl || exit 1
  done
done
cat $O/bucket.jsonl
