#!/bin/bash
# rocprofv3 kernel trace of latency-bound allreduces (2 processes, one GPU, hipGraph replay).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_latency" -o run -- python3 "$R/bench/latency_ipc.py" --nranks 2 --graph \
    --algos ll,oneshot --sizes 4,4096,65536 --iters 100 > "$R/gpurun_out/prof_latency.log" 2>&1) && echo "prof ok"
rc=$?; tail -8 gpurun_out/prof_latency.log; find gpurun_out/prof_latency -name "*kernel_stats.csv" | head; exit $rc
