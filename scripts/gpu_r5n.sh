#!/bin/bash
# Round 5, final tree: the driver's round-end order (whole GPU tier, smoke(), N = 1 bench), a kernel trace of the
# bench, and the 8-process self-launched shared-GPU rehearsal of bench.py once (per-rank phase logs and the crash
# report on). Every step bounded, chained.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5n
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5n
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/test_gpu_all.log 2>&1 && echo "gpu tests ok" && tail -1 $O/test_gpu_all.log || { tail -30 $O/test_gpu_all.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err && echo "profile ok" || exit 1
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n8.json 2> $O/bench_selflaunch_n8.err && echo "n=8 rehearsal ok" || { tail -40 $O/bench_selflaunch_n8.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_selflaunch_n8.json')); print(d['value'], d['unit'], d.get('bench_wall_s'), d['config']['algorithm'], json.dumps(d.get('readiness',{}).get('selftest_recovered')))"
