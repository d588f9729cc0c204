#!/bin/bash
# Round 4 A/B: the untyped executor held to 4 waves per SIMD (128 VGPRs, 10 spilled: two 512-thread
# workgroups per CU) with the group cap raised to 512 co-resident workgroups (abw/), against the library
# (138 VGPRs, one workgroup per CU). Ranks in one launch, 100 MiB per rank, interleaved, two repetitions.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4z
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4z
: > $O/ab.jsonl
for rep in 1 2; do
  for lib in main wpe4; do
    if [ $lib = wpe4 ]; then export FLEXAR_LIB_PATH=$R/abw/libflexar.so; else unset FLEXAR_LIB_PATH; fi
    for c in "4 flat+pull float32" "4 ring float32" "4 rhd+pull float32" "8 flat+pull float32" "4 flat+pull bfloat16"; do
      set -- $c
      echo -n "{\"lib\": \"$lib\", \"r\": " >> $O/ab.jsonl
      TEP_RANKS=$1 TEP_MIB=100 TEP_ITERS=10 timeout -k 10 120 python3 bench/typed_exec_probe.py $2 $3 >> $O/ab.jsonl || exit 1
      sed -i '$ s/$/}/' $O/ab.jsonl
    done
  done
done
cat $O/ab.jsonl
