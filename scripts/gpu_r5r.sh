#!/bin/bash
# Round 5, final tree after the packed fp8 reduction: the driver's round-end order (whole GPU tier, smoke(), N = 1
# bench) and a kernel trace of the bench. Every step bounded, chained.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5r
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5r
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/test_gpu_all.log 2>&1 && echo "gpu tests ok" && tail -1 $O/test_gpu_all.log || { tail -30 $O/test_gpu_all.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err && echo "profile ok" || exit 1
