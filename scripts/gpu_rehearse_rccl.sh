#!/bin/bash
# The driver's N>1 bench flow on a 1-GPU box with RCCL in it: "nccl" process group, RCCL reference and
# comparator, the '+rccl' message-transport tuner candidates (FLEXAR_BENCH_SHARED_RCCL=1 gives every rank
# its own NCCL_HOSTID, so RCCL accepts two ranks on one GPU and talks over loopback sockets). N=2 and N=4.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/rehearse_rccl_n2.log 2>&1 && echo "rehearse rccl n=2 ok" &&
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 10 --warmup 3 \
    > gpurun_out/rehearse_rccl_n4.log 2>&1 && echo "rehearse rccl n=4 ok"
rc=$?
tail -2 gpurun_out/rehearse_rccl_n2.log | cut -c1-1500; tail -2 gpurun_out/rehearse_rccl_n4.log 2>/dev/null | cut -c1-1500
exit $rc
