#!/bin/bash
# Multi-rank bench rehearsal on a 1-GPU box: N=2 and N=4 ranks sharing device 0 (gloo reference and
# barriers), exercising the tuner, the cost-model calibration and the JSON line the driver reads at N>1.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/rehearse_n2.log 2>&1 && echo "rehearse n=2 ok" &&
FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29503 bench.py --gpus 4 --steps 10 --warmup 3 \
    > gpurun_out/rehearse_n4.log 2>&1 && echo "rehearse n=4 ok"
rc=$?
tail -2 gpurun_out/rehearse_n2.log; tail -2 gpurun_out/rehearse_n4.log 2>/dev/null
exit $rc
