#!/bin/bash
# Round 4: fp32 partials vs per-hop rounding after the typed-layout changes (bf16, 100 MiB per rank, ranks in
# one launch), two repetitions.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4ag
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4ag
: > $O/partials.jsonl
for rep in 1 2; do
  for n in 4 8; do
    for spec in rhd+pull+f32 rhd+pull+rw ring+f32 ring+rw; do
      TEP_RANKS=$n TEP_MIB=100 TEP_ITERS=10 timeout -k 10 120 python3 bench/typed_exec_probe.py $spec bfloat16 >> $O/partials.jsonl || exit 1
    done
  done
done
cat $O/partials.jsonl
