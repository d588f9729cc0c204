#!/bin/bash
# Rehearse the driver's multi-rank bench flow (tuner, validation, rebuilds, JSON) with N ranks on ONE GPU.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_BENCH_SHARED_GPU=1
for n in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/rehearse_n$n.log 2>&1
  rc=$?
  echo "n=$n rc=$rc"; grep -E "tuner|metric|Error|error" gpurun_out/rehearse_n$n.log | tail -30
  [ $rc -eq 0 ] || exit $rc
done
