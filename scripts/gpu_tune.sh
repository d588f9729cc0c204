#!/bin/bash
# Rehearse the measured tune-table tool with 4 ranks on one GPU, then check `auto` follows the table.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_BENCH_SHARED_GPU=1
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29511 tools/flexar_tune.py --min-bytes 4K --max-bytes 16M --out gpurun_out/tune_shared4.txt \
    --jsonl gpurun_out/tune_shared4.jsonl > gpurun_out/tune.log 2>&1
rc=$?; grep -E "\[tune\]|tune_file|Error" gpurun_out/tune.log | tail -20; cat gpurun_out/tune_shared4.txt
exit $rc
