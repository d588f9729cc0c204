#!/bin/bash
# Round 6, first GPU pass: link-balanced multi-channel trees (LocalGroup bit-exactness, all algorithms,
# typed partials), lifecycle (teardown agreed over the bootstrap without a host page), MPI zero copy by
# default, the shared-GPU acceptance matrix, then a short N=1 bench. Each step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6a
export FLEXAR_NO_BUILD=1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gpu_kernels.py -k "channelled or all_algorithms or typed_fp32 or dtypes" \
    > gpurun_out/r6a/kernels.log 2>&1 && echo "kernels ok" &&
timeout -k 10 600 $PYT tests/test_gpu_lifecycle.py > gpurun_out/r6a/lifecycle.log 2>&1 && echo "lifecycle ok" &&
timeout -k 10 600 $PYT tests/test_gpu_mpi.py > gpurun_out/r6a/mpi.log 2>&1 && echo "mpi ok" &&
timeout -k 10 900 $PYT tests/test_gpu_multidevice.py > gpurun_out/r6a/multidevice.log 2>&1 && echo "multidevice ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6a/bench_n1.log 2>&1 && echo "bench ok"
rc=$?
for f in gpurun_out/r6a/*.log; do echo "== $f"; tail -4 "$f" | cut -c1-400; done
exit $rc
