#!/bin/bash
# Kernel + group GPU tests only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=5000
timeout -k 10 600 python3 -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/kernels_tests.log 2>&1; rc=$?
tail -15 gpurun_out/kernels_tests.log
exit $rc
