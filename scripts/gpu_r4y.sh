#!/bin/bash
# Round 4: kernel trace of the DDP step with the fp8 and the MX gradient hooks (2 ranks sharing the GPU):
# where does the MX hook's in-step time go? One bounded rocprofv3 run (kernel trace + stats only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4y
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r4y
for m in fp8hook mxhook; do
  DDPB_RANKS=2 DDPB_MODES=$m DDPB_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv \
      -- python3 bench/ddp_step_bench.py > $O/ddp_$m.jsonl 2> $O/ddp_$m.err || exit 1
  echo "$m ok"
done
