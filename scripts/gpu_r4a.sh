#!/bin/bash
# Round 4, first GPU pass: smoke, the new lifecycle tests (collective close, named self-test HIP errors,
# the agreed retry), misaligned caller buffers on the vector path (test + A/B), the calibration tests (the
# driver's round-3 failure), then the whole GPU tier. Each GPU step has its own time limit; steps chained
# with && (the first failure ends the call).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lifecycle.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/test_gpu_lifecycle.log 2>&1 && echo "lifecycle tests ok" &&
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_kernels.py -x -v -k misaligned --timeout 120 --timeout-method thread \
    > gpurun_out/test_gpu_misaligned.log 2>&1 && echo "misaligned tests ok" &&
timeout -k 10 120 python3 bench/misaligned_bench.py > gpurun_out/misaligned_vector.jsonl 2> gpurun_out/misaligned_vector.err &&
FLEXAR_SCALAR_MISALIGNED=1 timeout -k 10 120 python3 bench/misaligned_bench.py > gpurun_out/misaligned_scalar.jsonl \
    2> gpurun_out/misaligned_scalar.err && echo "misaligned bench ok" &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_calibration.py -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/test_gpu_calibration.log 2>&1 && echo "calibration tests ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > gpurun_out/test_gpu_all.log 2>&1 && echo "gpu tests ok"
rc=$?
tail -5 gpurun_out/test_gpu_lifecycle.log; tail -3 gpurun_out/test_gpu_misaligned.log 2>/dev/null
tail -3 gpurun_out/test_gpu_calibration.log 2>/dev/null; tail -3 gpurun_out/test_gpu_all.log 2>/dev/null
exit $rc
