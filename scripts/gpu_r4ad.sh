#!/bin/bash
# Round 4: reduce-scatter with and without the MX wire (4 and 8 ranks in one launch; 25 and 100 MiB of input
# per rank).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4ad
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4ad
: > $O/rs.jsonl
for n in 4 8; do
  for mib in 25 100; do
    for c in "flat float32" "flat+mxe4m3 float32" "flat bfloat16" "flat+mxe4m3 bfloat16"; do
      set -- $c
      TEP_COLL=reduce_scatter TEP_RANKS=$n TEP_MIB=$mib TEP_ITERS=20 timeout -k 10 120 python3 bench/typed_exec_probe.py $1 $2 >> $O/rs.jsonl || exit 1
    done
  done
done
cat $O/rs.jsonl
