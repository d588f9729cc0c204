#!/bin/bash
# Round 6: the MPI zero-copy tests (refused registrations remembered per buffer) and the channelled-tree kernels on
# the current library. Each step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6f
export FLEXAR_NO_BUILD=1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_mpi.py > gpurun_out/r6f/mpi.log 2>&1 && echo "mpi ok" &&
timeout -k 10 600 $PYT tests/test_gpu_kernels.py -k "channelled or all_algorithms" > gpurun_out/r6f/kernels.log 2>&1 && echo "kernels ok"
rc=$?
for f in gpurun_out/r6f/*.log; do echo "== $f"; tail -3 "$f" | cut -c1-300; done
exit $rc
