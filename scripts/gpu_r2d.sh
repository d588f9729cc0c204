#!/bin/bash
# Round 2: pipelined copy-engine allreduce (group pieces, IPC processes), then the whole tier and the
# dma bench (bf16 1 GiB, config #3) on the shared-GPU rehearsal.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ipc.py -x -v -k "dma or randomized or mixed" \
    --timeout 120 --timeout-method thread > gpurun_out/r2d_dma.log 2>&1 && echo "dma ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/r2d_gpu_all.log 2>&1 && echo "gpu tests ok" &&
FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 5 --warmup 2 --dtype bfloat16 --size-mb 1024 \
    --algo dma --no-small > gpurun_out/r2d_dma_bf16_1g.log 2>&1 && echo "dma bench ok"
rc=$?
tail -3 gpurun_out/r2d_dma.log; tail -3 gpurun_out/r2d_gpu_all.log; tail -1 gpurun_out/r2d_dma_bf16_1g.log
exit $rc
