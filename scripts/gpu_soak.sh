#!/bin/bash
# Soak: the randomized collective sequence (tests/test_gpu_ipc.py _stress_worker) at 600 calls per run, N = 4,
# N = 8 and N = 4 with a delayed peer, every rank on one GPU, every result exact. One bounded pytest run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_SOAK="${FLEXAR_SOAK:-600}"
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_ipc.py -x -v -k "soak or rebuild_cycles" --timeout 950 --timeout-method thread \
    > gpurun_out/soak.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/soak.log | tail -8
exit $rc
