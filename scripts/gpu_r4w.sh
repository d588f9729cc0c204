#!/bin/bash
# Round 4: the self-launched 8-process shared-GPU bench rehearsal on the final tree (config #5 with the MX
# wire at 8 ranks). One bounded step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4w
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4w
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n8.json 2> $O/bench_selflaunch_n8.err && echo "n=8 ok"
rc=$?
python3 -c "import json; d=json.load(open('$O/bench_selflaunch_n8.json')); print(d['value'], json.dumps(d.get('config5')), d.get('bench_wall_s'))" || true
exit $rc
