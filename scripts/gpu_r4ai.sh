#!/bin/bash
# Round 4, final GPU pass (native MX codec): the driver's round-end order on the current tree - the whole GPU tier, smoke(),
# the N = 1 bench - then a kernel-trace profile of the N = 1 bench. Each GPU step bounded; chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4ai
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r4ai
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/test_gpu_all.log 2>&1 && echo "gpu tests ok" &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err && echo "profile ok"
rc=$?
tail -3 $O/test_gpu_all.log 2>/dev/null
exit $rc
