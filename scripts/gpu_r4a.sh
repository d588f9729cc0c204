#!/bin/bash
# Round 4, first GPU pass: smoke, the new lifecycle tests (collective close, named self-test HIP errors,
# the agreed retry), the calibration tests (the driver's round-3 failure), then the whole GPU tier. Each
# GPU step has its own time limit; steps chained with && (the first failure ends the call).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lifecycle.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/test_gpu_lifecycle.log 2>&1 && echo "lifecycle tests ok" &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_calibration.py -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/test_gpu_calibration.log 2>&1 && echo "calibration tests ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > gpurun_out/test_gpu_all.log 2>&1 && echo "gpu tests ok"
rc=$?
tail -5 gpurun_out/test_gpu_lifecycle.log; tail -3 gpurun_out/test_gpu_calibration.log 2>/dev/null
tail -3 gpurun_out/test_gpu_all.log 2>/dev/null
exit $rc
