#!/bin/bash
# Round 6: smoke and the whole GPU test tier on the current tree (what the driver runs at round end), then the
# N=1 bench. Each step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6_tier
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/r6_tier/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread \
    > gpurun_out/r6_tier/test_gpu_all.log 2>&1 && echo "gpu tests ok" &&
timeout -k 10 300 python3 bench.py > gpurun_out/r6_tier/bench_n1.log 2>&1 && echo "bench ok"
rc=$?
tail -3 gpurun_out/r6_tier/test_gpu_all.log; tail -1 gpurun_out/r6_tier/bench_n1.log | cut -c1-400
exit $rc
