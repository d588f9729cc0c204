#!/bin/bash
# zero-copy push variant: group tests, IPC processes, microbench, bench rehearsal N=2/4
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ipc.py -x -v -m gpu --timeout 180 \
    --timeout-method thread -k "all_algorithms or zero_copy" > gpurun_out/test_zc2.log 2>&1 && echo "zc tests ok" &&
timeout -k 10 300 python3 bench/zc_bench.py > gpurun_out/zc_bench.jsonl 2> gpurun_out/zc_bench.err && echo "zc bench ok" &&
bash scripts/gpu_rehearse.sh
rc=$?
tail -2 gpurun_out/test_zc2.log
exit $rc
