#!/bin/bash
# Small-message latency, 2 and 4 processes on one GPU. Extra args go to bench/latency_ipc.py (e.g. --graph).
# OUT names the results file under gpurun_out/ (default latency_ipc.jsonl).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
OUT="gpurun_out/${OUT:-latency_ipc.jsonl}"
rm -f "$OUT"
timeout -k 10 300 python bench/latency_ipc.py --nranks 2 --out "$OUT" "$@" > gpurun_out/latency2.log 2>&1 && echo "lat2 ok" &&
timeout -k 10 300 python bench/latency_ipc.py --nranks 4 --out "$OUT" "$@" > gpurun_out/latency4.log 2>&1 && echo "lat4 ok"
rc=$?; cat "$OUT"; exit $rc
