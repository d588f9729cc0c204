#!/bin/bash
# Round 5: after the reduction's grid-interleaved form and the wide unroll became the default - the kernel tests,
# the N = 1 bench (reduce_kernel section) and its kernel trace. Bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5h
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5h
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu --timeout 240 --timeout-method thread \
    > $O/tests.log 2>&1 && echo "kernel tests ok" && tail -1 $O/tests.log &&
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err && echo "profile ok"
