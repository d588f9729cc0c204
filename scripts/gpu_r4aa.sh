#!/bin/bash
# Round 4: the c10d backend's FLEXAR_PG_COMPRESS option in a DDP run (2 ranks, one GPU) and the hook tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4aa
export FLEXAR_NO_BUILD=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_backend.py -x -v -k "ddp_over_flexar" --timeout 240 --timeout-method thread \
    > gpurun_out/r4aa/test_backend.log 2>&1
rc=$?
tail -n 14 gpurun_out/r4aa/test_backend.log
exit $rc
