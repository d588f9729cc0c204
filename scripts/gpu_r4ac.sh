#!/bin/bash
# Round 4: the backend's compressed reduce-scatter, plus the backend collective / FSDP2 tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4ac
export FLEXAR_NO_BUILD=1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_backend.py -x -v -k "compressed or reduce_scatter or fsdp2 or functional or backend_mx" \
    --timeout 240 --timeout-method thread > gpurun_out/r4ac/test_backend.log 2>&1
rc=$?
tail -n 12 gpurun_out/r4ac/test_backend.log
exit $rc
