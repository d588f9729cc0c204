#!/bin/bash
# Round 4: DDP step with compressed gradients - plain hook vs global-scale fp8 hook vs OCP MX hook, GPT-small,
# 2 and 4 ranks sharing one GPU (bench/ddp_step_bench.py). Each run bounded.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4x
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4x
DDPB_RANKS=2 DDPB_MODES=hook,fp8hook,mxhook timeout -k 10 400 python3 bench/ddp_step_bench.py > $O/ddp_n2.jsonl 2> $O/ddp_n2.err && echo "n2 ok" &&
DDPB_RANKS=4 DDPB_MODES=hook,fp8hook,mxhook timeout -k 10 500 python3 bench/ddp_step_bench.py > $O/ddp_n4.jsonl 2> $O/ddp_n4.err && echo "n4 ok"
rc=$?
cat $O/ddp_n2.jsonl $O/ddp_n4.jsonl 2>/dev/null
exit $rc
