#!/bin/bash
# bench.py's final-check fallback chain: the N=1 line, and a shared-GPU N=2 run (RCCL over loopback) whose
# tuner pick is rejected on purpose (FLEXAR_BENCH_REJECT_FIRST=1): the next-fastest candidate must take over
# on a fresh communicator and the JSON line must name the rejection.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 bench.py > gpurun_out/fb_n1.log 2>&1 && echo "n1 ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 FLEXAR_BENCH_REJECT_FIRST=1 timeout -k 10 400 \
    python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-calibrate > gpurun_out/fb_n2.log 2>&1 && echo "n2 fallback ok"
rc=$?
tail -1 gpurun_out/fb_n1.log | cut -c1-300; grep -E "trying the next|running" gpurun_out/fb_n2.log; tail -1 gpurun_out/fb_n2.log | cut -c1-600
exit $rc
