#!/bin/bash
# Round 3, first GPU pass: smoke, the new calibration / probe-agreement GPU tests, then the whole GPU tier
# (the comm.hip split and the program-priced selector touch every path), then the driver's N=2 flow with
# RCCL on one GPU. Each GPU step has its own time limit; steps chained with && (the first failure ends it).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_calibration.py -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/test_gpu_calibration.log 2>&1 && echo "calibration tests ok" &&
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > gpurun_out/test_gpu_all.log 2>&1 && echo "gpu tests ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/rehearse_rccl_n2.log 2>&1 && echo "rehearse n=2 ok"
rc=$?
tail -3 gpurun_out/test_gpu_calibration.log; tail -3 gpurun_out/test_gpu_all.log 2>/dev/null
tail -1 gpurun_out/rehearse_rccl_n2.log 2>/dev/null | cut -c1-3000
exit $rc
