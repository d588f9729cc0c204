#!/bin/bash
# Round 3, after the typed-executor rework: smoke, the whole GPU tier, then the driver's N=4 flow on one GPU
# with RCCL (config #3 rhd bf16 +f32 / +rw, config #5 fp8 run through the typed executors). Each GPU step has
# its own time limit; steps chained with && (the first failure ends it).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > gpurun_out/test_gpu_all.log 2>&1 && echo "gpu tests ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 10 --warmup 3 \
    > gpurun_out/rehearse_rccl_n4.log 2>&1 && echo "rehearse n=4 ok"
rc=$?
tail -3 gpurun_out/test_gpu_all.log 2>/dev/null
tail -1 gpurun_out/rehearse_rccl_n4.log 2>/dev/null | cut -c1-2000
exit $rc
