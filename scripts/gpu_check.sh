#!/bin/bash
# First-light GPU check: smoke, kernel/group tests, N=1 bench, IPC tests. Each GPU step bounded.
set -o pipefail
mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
echo "== rocminfo" ; (rocm-smi --showproductname 2>&1 | head -20) > gpurun_out/smi.log
timeout -k 10 400 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/test_gpu_kernels.log 2>&1 && echo "kernels ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1 && echo "bench ok" &&
timeout -k 10 400 python -m pytest tests/test_gpu_ipc.py -x -q > gpurun_out/test_gpu_ipc.log 2>&1 && echo "ipc ok"
rc=$?
tail -5 gpurun_out/*.log
exit $rc
