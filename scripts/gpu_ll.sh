#!/bin/bash
# LL protocol check after a kernel change: numerics tests, then latency eager + graph (2 processes, one GPU).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_faults.py tests/test_gpu_ipc.py > gpurun_out/pytest_ll.txt 2>&1 && echo tests_ok &&
timeout -k 10 200 python bench/latency_ipc.py --nranks 2 --algos ll,oneshot,oneshot+wt --out gpurun_out/lat_ll_eager.jsonl > gpurun_out/lat_ll1.txt 2>&1 && echo eager_ok &&
timeout -k 10 200 python bench/latency_ipc.py --nranks 2 --graph --algos ll,oneshot,oneshot+wt --out gpurun_out/lat_ll_graph.jsonl > gpurun_out/lat_ll2.txt 2>&1 && echo graph_ok &&
timeout -k 10 200 python bench/latency_ipc.py --nranks 4 --graph --algos ll,oneshot,oneshot+wt --out gpurun_out/lat_ll_graph.jsonl > gpurun_out/lat_ll3.txt 2>&1 && echo graph4_ok
rc=$?; tail -3 gpurun_out/pytest_ll.txt; exit $rc
