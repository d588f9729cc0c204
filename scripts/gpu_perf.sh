#!/bin/bash
# Kernel microbenchmarks + rocprofv3 kernel-trace stats on one MI355X.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
timeout -k 10 600 python bench/kernel_bench.py --out gpurun_out/kernel_bench.jsonl > gpurun_out/kernel_bench.log 2>&1 && echo "kernel_bench ok" &&
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_kernels" -o run -- python3 "$R/bench/kernel_bench.py" --what reduce,copy > "$R/gpurun_out/prof_kernels.log" 2>&1 ) && echo "rocprof ok"
rc=$?
tail -n 3 gpurun_out/kernel_bench.log
exit $rc
