#!/bin/bash
# Copy-engine (dma) allreduce + +wt protocol: kernel and IPC GPU tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=5000
timeout -k 10 600 python3 -m pytest tests/test_gpu_kernels.py tests/test_gpu_ipc.py -x -q -m gpu > gpurun_out/dma_tests.log 2>&1; rc=$?
tail -15 gpurun_out/dma_tests.log
exit $rc
