#!/bin/bash
# Round 6: bench JSON contract on GPU (registered auto choice via last_spec), MPI zero copy after the call-memo
# change, zero-copy IPC tests. Each step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6g
export FLEXAR_NO_BUILD=1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_gpu_bench.py > gpurun_out/r6g/bench.log 2>&1 && echo "bench tests ok" &&
timeout -k 10 600 $PYT tests/test_gpu_mpi.py > gpurun_out/r6g/mpi.log 2>&1 && echo "mpi ok" &&
timeout -k 10 600 $PYT tests/test_gpu_ipc.py -k "zc or zero or reg" > gpurun_out/r6g/ipc.log 2>&1 && echo "ipc ok"
rc=$?
for f in gpurun_out/r6g/*.log; do echo "== $f"; tail -3 "$f" | cut -c1-300; done
exit $rc
