#!/bin/bash
# Round-end rehearsal: smoke, the whole GPU test tier, the N=1 bench and a rocprofv3 kernel-stats run
# of the bench. Each GPU step has its own time limit; the steps are chained with && so the first
# failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/test_gpu_all.log 2>&1 && echo "gpu tests ok" &&
timeout -k 10 300 python3 bench.py > gpurun_out/bench_n1.log 2>&1 && echo "bench ok" &&
FLEXAR_BENCH_SHARED_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/rehearse_n2.log 2>&1 && echo "rehearse n=2 ok" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench" \
    -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/gpurun_out/prof_bench.log" 2>&1) && echo "prof ok"
rc=$?
tail -3 gpurun_out/test_gpu_all.log; tail -2 gpurun_out/bench_n1.log
exit $rc
