#!/bin/bash
# Round 3: the lane-interleaved typed executor - its GPU numerics tests (fp32 partials within 1 ulp, fp8 wire
# bit-exact against the torch emulation), then the efficiency probe again.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
rm -rf gpurun_out/typed_probe
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_typed_staging.py -x -q --timeout 240 \
    --timeout-method thread > gpurun_out/r3e_tests.log 2>&1 && echo "kernel tests ok" &&
bash scripts/gpu_typed_probe.sh
rc=$?
tail -3 gpurun_out/r3e_tests.log
exit $rc
