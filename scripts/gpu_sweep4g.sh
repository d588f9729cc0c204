#!/bin/bash
# BASELINE config #4's full range: the cost-model ("auto") choice for every size 4 KiB .. 4 GiB (x4 steps),
# 2 ranks sharing one GPU (gloo reference; shared HBM, not xGMI). The 1 and 4 GiB points take several
# workspace pieces per call (size_t counts, piece loop).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/sweep4g
export FLEXAR_NO_BUILD=1 FLEXAR_BENCH_SHARED_GPU=1
rm -f gpurun_out/sweep4g/sweep.jsonl
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29620 bench.py --gpus 2 --size-mb 4 --no-tune --no-calibrate --steps 5 --warmup 2 \
    --sweep 4K:4G --sweep-out gpurun_out/sweep4g/sweep.jsonl > gpurun_out/sweep4g/run.log 2>&1 && echo "sweep ok"
rc=$?
cat gpurun_out/sweep4g/sweep.jsonl 2>/dev/null | cut -c1-200
exit $rc
