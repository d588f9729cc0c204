#!/bin/bash
# Zero-copy ("+zc") checks: the group tests (every schedule and collective incl. the +zc forms), the
# multi-process registered-buffer tests (collectives, automatic choice, HIP graph, randomized sequence), DDP
# with zero-copy gradient buckets and the MPI layer's collective registration.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ipc.py tests/test_gpu_backend.py \
    tests/test_gpu_mpi.py -x -v -m gpu --timeout 180 --timeout-method thread \
    -k "all_algorithms or reduce_scatter or all_to_all or broadcast or zero_copy or captured or randomized or ddp or mpi" \
    > gpurun_out/test_zc.log 2>&1 && echo "zc tests ok"
rc=$?
tail -3 gpurun_out/test_zc.log
exit $rc
