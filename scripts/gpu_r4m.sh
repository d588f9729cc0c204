#!/bin/bash
# Round 4, twelfth GPU pass: the MX DDP hook (2 ranks, against a single-process reference), then the
# self-launched 4- and 8-rank bench rehearsals whose config #5 section now times the MX wire next to the
# global-scale one. Each GPU step bounded; chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4m
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4m
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_backend.py -x -v -k "hook" --timeout 240 --timeout-method thread \
    > $O/test_hooks.log 2>&1 && echo "hook tests ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 400 python3 bench.py --gpus 4 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n4.json 2> $O/bench_selflaunch_n4.err && echo "n=4 ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n8.json 2> $O/bench_selflaunch_n8.err && echo "n=8 ok"
rc=$?
tail -n 3 $O/test_hooks.log
python3 - <<'PY'
import json
for n in (4, 8):
    try:
        d = json.load(open(f"gpurun_out/r4m/bench_selflaunch_n{n}.json"))
        print(n, d["value"], json.dumps(d.get("config5")), d.get("bench_wall_s"))
    except Exception as e:
        print(n, "no result", e)
PY
exit $rc
