#!/bin/bash
# Round 4, sixth GPU pass: the semantics of gfx950's scaled fp8 conversions (bin/scaled_cvt_probe), the N = 8
# self-launched bench rehearsal with the hardware-queue cap now applied over the box's explicit default, and
# the whole GPU tier. Each GPU step bounded; chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4f
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4f
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
timeout -k 10 60 ./bin/scaled_cvt_probe > $O/scaled_cvt_probe.jsonl && cat $O/scaled_cvt_probe.jsonl &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n8.json 2> $O/bench_selflaunch_n8.err && echo "self-launch n=8 ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/test_gpu_all.log 2>&1 && echo "gpu tests ok"
rc=$?
tail -3 $O/test_gpu_all.log 2>/dev/null
exit $rc
