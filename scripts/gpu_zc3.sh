#!/bin/bash
# zero-copy collectives: group tests (RS/AG/A2A/bcast) and the multi-process registered buffer test
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ipc.py -x -v -m gpu --timeout 180 \
    --timeout-method thread -k "reduce_scatter or all_to_all or broadcast or zero_copy or all_algorithms" \
    > gpurun_out/test_zc3.log 2>&1 && echo "zc collective tests ok"
rc=$?
tail -3 gpurun_out/test_zc3.log
exit $rc
