#!/bin/bash
# Round 5: the driver's round-end order on the current tree - the whole GPU tier, smoke(), the N = 1 bench -
# each step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5d
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5d
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/test_gpu_all.log 2>&1 && echo "gpu tests ok" &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json
rc=$?
tail -3 $O/test_gpu_all.log 2>/dev/null
exit $rc
