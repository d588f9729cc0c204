#!/bin/bash
# Changed GPU tests (stale-staging hand-off, IPC connect agreement, backend), the multi-rank bench flow
# rehearsed on one GPU (N=2,4), the N=1 bench and a rocprofv3 kernel-stats run. Each GPU step bounded,
# chained with && so the first failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_faults.py tests/test_gpu_ipc.py tests/test_gpu_backend.py \
    tests/test_gpu_multidevice.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/t_changed.log 2>&1 \
  && echo "changed tests ok" &&
for n in 2 4; do
  FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 \
      > gpurun_out/rehearse_n$n.log 2>&1 || exit $?
  echo "rehearse n=$n ok"
done &&
timeout -k 10 300 python3 bench.py > gpurun_out/bench_n1.log 2>&1 && echo "bench ok" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_bench" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 \
    > "$R/gpurun_out/prof_bench.log" 2>&1) && echo "prof ok"
rc=$?
tail -3 gpurun_out/t_changed.log; tail -1 gpurun_out/bench_n1.log
exit $rc
