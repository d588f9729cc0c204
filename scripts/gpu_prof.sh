#!/bin/bash
# GPU tests + kernel microbench + rocprofv3 HBM counters (FETCH_SIZE / WRITE_SIZE in separate passes).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
[ -n "$SKIP_TESTS" ] || { timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok"; } || { echo "pytest gpu FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 600 python bench/kernel_bench.py --out gpurun_out/kernel_bench.jsonl > gpurun_out/kernel_bench.log 2>&1 && echo "kernel_bench ok" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$c" -o run -- python3 "$R/bench/kernel_bench.py" --what reduce --dtypes float32,bfloat16 --fanins 1,2,8 --iters 3 > "$R/gpurun_out/pmc_$c.log" 2>&1 ) && echo "pmc $c ok" || { echo "pmc $c failed"; exit 1; }
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1 && echo "bench ok" && tail -1 gpurun_out/bench_n1.log
