#!/bin/bash
# Validate the write-through protocol (+wt) on the GPU, then compare per-kernel protocol cost.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 900 python3 -m pytest tests/test_gpu_kernels.py tests/test_gpu_ipc.py -x -q -m gpu > gpurun_out/wt_tests.log 2>&1 && echo "tests ok" && \
bash scripts/gpu_probe.sh --specs "ll,oneshot,oneshot+wt,flat+pull,flat+pull+wt,flat+push+wt,ring,ring+wt" --grids "4,8,16,32"
