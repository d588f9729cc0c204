#!/bin/bash
# The driver's multi-rank bench path rehearsed with N ranks sharing one GPU (N=2,4): torch.distributed.run,
# tuner, RCCL cross-check, JSON line. Each step bounded; the first failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
for n in 2 4; do
  FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 10 --warmup 3 \
      > gpurun_out/rehearse_n$n.log 2>&1 || exit $?
  echo "rehearse n=$n ok"; tail -1 gpurun_out/rehearse_n$n.log
done
