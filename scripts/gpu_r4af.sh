#!/bin/bash
# Round 4: MX group tests incl. the default-spec wire handling and kernel_info of every executor class.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4af
export FLEXAR_NO_BUILD=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mx.py tests/test_gpu_kernels.py -x -v -k "mx or kernel_info or default_spec or fp8" \
    --timeout 240 --timeout-method thread > gpurun_out/r4af/test_mx.log 2>&1
rc=$?
tail -n 6 gpurun_out/r4af/test_mx.log
exit $rc
