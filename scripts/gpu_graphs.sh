#!/bin/bash
# Captured-allreduce test and the tensor-parallel decode example (eager vs one hipGraph), ranks sharing one GPU.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
rm -f gpurun_out/tp_decode.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ipc.py -k "captured or graph or memo" \
    > gpurun_out/pytest_graphs.txt 2>&1 && echo tests_ok &&
timeout -k 10 300 python examples/tp_decode.py --nranks 2 --out gpurun_out/tp_decode.jsonl > gpurun_out/tp2.txt 2>&1 && echo tp2_ok &&
timeout -k 10 300 python examples/tp_decode.py --nranks 4 --out gpurun_out/tp_decode.jsonl > gpurun_out/tp4.txt 2>&1 && echo tp4_ok
rc=$?; tail -4 gpurun_out/pytest_graphs.txt; cat gpurun_out/tp_decode.jsonl 2>/dev/null; tail -5 gpurun_out/tp2.txt; exit $rc
