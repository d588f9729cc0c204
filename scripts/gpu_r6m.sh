#!/bin/bash
# Round 6: the randomized collective stress (80 calls, the regular tier's form) and the soak (600 calls per run,
# N = 4, N = 8 and N = 4 with a delayed peer) with the channelled trees in the mix, every result exact.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6m
export FLEXAR_NO_BUILD=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ipc.py -x -v -k "randomized" --timeout 350 --timeout-method thread \
    > gpurun_out/r6m/stress.log 2>&1 && echo "stress ok" &&
FLEXAR_SOAK=600 timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_ipc.py -x -v -k "soak or rebuild_cycles" --timeout 950 \
    --timeout-method thread > gpurun_out/r6m/soak.log 2>&1 && echo "soak ok"
rc=$?
grep -hE "PASSED|FAILED|passed|failed" gpurun_out/r6m/*.log | tail -12
exit $rc
