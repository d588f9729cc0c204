#!/bin/bash
# BASELINE config #3 buffer (bf16, 1 GiB per rank) on 4 ranks sharing one GPU
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
FLEXAR_LOG_LEVEL=info FLEXAR_BENCH_TRACEBACK_S=60 FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29505 bench.py --gpus 4 --steps 10 --warmup 3 \
    --dtype bfloat16 --size-mb 1024 > gpurun_out/cfg3_bf16_1g_n4.log 2>&1 && echo "cfg3 ok"
rc=$?
tail -1 gpurun_out/cfg3_bf16_1g_n4.log | cut -c1-600
exit $rc
