#!/bin/bash
# Round 5, final tree: the 8-process self-launched shared-GPU rehearsal of bench.py once (per-rank phase logs and
# the crash report on; RCCL over loopback). Bounded.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5s
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5s
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n8.json 2> $O/bench_selflaunch_n8.err && echo "n=8 rehearsal ok" || { tail -40 $O/bench_selflaunch_n8.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_selflaunch_n8.json')); print(d['value'], d['unit'], d.get('bench_wall_s'), d['config']['algorithm'], json.dumps(d.get('readiness',{}).get('selftest_recovered')), json.dumps(d.get('config5'))[:400])"
