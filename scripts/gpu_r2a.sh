#!/bin/bash
# Round 2: readiness gate (probe + self-test + downgrade) on one GPU, then the whole GPU tier and the
# shared-GPU bench rehearsal with the new reporting fields.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ipc.py -x -v -k readiness --timeout 120 --timeout-method thread \
    > gpurun_out/r2a_readiness.log 2>&1 && echo "readiness ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/r2a_gpu_all.log 2>&1 && echo "gpu tests ok" &&
FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/r2a_rehearse_n2.log 2>&1 && echo "rehearse n=2 ok" &&
timeout -k 10 300 python3 bench.py > gpurun_out/r2a_bench_n1.log 2>&1 && echo "bench ok"
rc=$?
tail -3 gpurun_out/r2a_gpu_all.log; tail -1 gpurun_out/r2a_rehearse_n2.log
exit $rc
