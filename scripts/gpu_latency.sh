#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
rm -f gpurun_out/latency_ipc.jsonl
timeout -k 10 300 python bench/latency_ipc.py --nranks 2 --out gpurun_out/latency_ipc.jsonl > gpurun_out/latency2.log 2>&1 && echo "lat2 ok" &&
timeout -k 10 300 python bench/latency_ipc.py --nranks 4 --out gpurun_out/latency_ipc.jsonl > gpurun_out/latency4.log 2>&1 && echo "lat4 ok"
rc=$?; cat gpurun_out/latency_ipc.jsonl; exit $rc
