#!/bin/bash
# Round-end rehearsal: the whole GPU test tier, smoke, and the N=1 bench. Each GPU step bounded.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 900 python3 -m pytest tests -x -q -m gpu > gpurun_out/test_gpu_all.log 2>&1 && echo "gpu tests ok" &&
timeout -k 10 300 python3 bench.py > gpurun_out/bench_n1.log 2>&1 && echo "bench ok"
rc=$?
tail -3 gpurun_out/test_gpu_all.log; tail -2 gpurun_out/bench_n1.log
exit $rc
