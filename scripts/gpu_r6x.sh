#!/bin/bash
# One-off: the multi-device acceptance matrix at world 8 with every rank on device 0 (the regular tier runs 2 and
# 4 shared), so the per-process fan-in-8 executors - untyped, fp8 and MX wires (2-destination form) - are checked
# for exactness on the final tree. 8 processes: 2 hardware queues each (see gpu_r6_n8.sh).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6x
export FLEXAR_NO_BUILD=1 GPU_MAX_HW_QUEUES=2
timeout -k 10 900 python3 -u scripts/matrix_n8.py > gpurun_out/r6x/matrix_n8.log 2>&1
rc=$?
tail -5 gpurun_out/r6x/matrix_n8.log
exit $rc
