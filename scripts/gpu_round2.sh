#!/bin/bash
# Full GPU test suite + cache-policy variant microbenchmarks + N=1 bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" || { echo "pytest gpu FAILED"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
for v in "" _ntl _nts _ntb; do
  if [ -z "$v" ]; then d="$R/allreduce_over_mpi_amd/_lib"; else d="$R/allreduce_over_mpi_amd/_lib$v"; fi
  FLEXAR_LIB_DIR="$d" timeout -k 10 300 python bench/kernel_bench.py --what reduce,copy --out gpurun_out/kb_variant${v:-_base}.jsonl > gpurun_out/kb_variant${v:-_base}.log 2>&1 || { echo "variant $v failed"; exit 1; }
done
echo "variants ok"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1 && echo "bench ok" && tail -1 gpurun_out/bench_n1.log
