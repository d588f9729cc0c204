#!/bin/bash
# Round 2: message transport (RCCL resolved at run time, single-rank device path), then the whole GPU tier.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_msg.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r2c_msg.log 2>&1 && echo "msg ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/r2c_gpu_all.log 2>&1 && echo "gpu tests ok"
rc=$?
tail -3 gpurun_out/r2c_msg.log; tail -3 gpurun_out/r2c_gpu_all.log
exit $rc
