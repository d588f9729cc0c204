#!/bin/bash
# Round 5, first pass: the new readiness / host-page / breadcrumb GPU tests, then the N = 1 bench with its new
# reduce_kernel section and a kernel-trace profile of the same run. Each GPU step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5a
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5a
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_bench.py tests/test_gpu_kernels.py -x -v -m gpu \
    --timeout 240 --timeout-method thread > $O/tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err && echo "profile ok"
rc=$?
tail -5 $O/tests.log 2>/dev/null
exit $rc
