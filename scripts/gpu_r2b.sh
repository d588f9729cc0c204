#!/bin/bash
# Round 2: typed staging on the device (fp32 partials, fp8 wire with fused scales), then the whole tier.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -v -k "typed or fp8_wire or dtypes" --timeout 120 \
    --timeout-method thread > gpurun_out/r2b_typed.log 2>&1 && echo "typed ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/r2b_gpu_all.log 2>&1 && echo "gpu tests ok"
rc=$?
tail -3 gpurun_out/r2b_typed.log; tail -3 gpurun_out/r2b_gpu_all.log
exit $rc
