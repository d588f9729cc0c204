#!/bin/bash
# The driver's N = 8 bench flow on a 1-GPU box: 8 ranks on device 0, "nccl" process group with one
# NCCL_HOSTID per rank (RCCL over loopback sockets), default arguments (budget 400 s), so the N = 8 tuner
# candidates (full-mesh ring:7, trees 2,4 / 4,2, RHD, typed partials) and every config section run once
# before the driver's 8-GPU run. One GPU step, bounded; the summary is printed from the JSON line.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6_n8
export FLEXAR_NO_BUILD=1 FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1
# 8 processes x the default 4 hardware queues oversubscribe the GPU's compute queues: the command processor
# then time-slices the processes and every cross-rank hand-off waits for a queue switch (~12 ms per call)
export GPU_MAX_HW_QUEUES="${REHEARSE_HW_QUEUES:-2}"
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 10 --warmup 3 \
    > gpurun_out/r6_n8/rehearse_rccl_n8.log 2>&1 && echo "rehearse rccl n=8 ok"
rc=$?
grep '^{' gpurun_out/r6_n8/rehearse_rccl_n8.log > gpurun_out/r6_n8/bench_shared_rccl_n8.json 2>/dev/null
python3 - <<'PY' 2>/dev/null
import json
d = json.load(open("gpurun_out/r6_n8/bench_shared_rccl_n8.json"))
print("value", d["value"], "alg", d["config"]["algorithm"], "wall", d["bench_wall_s"], "dropped", d["dropped"])
print("tuner", json.dumps(d["tuner"])[:1500])
print("cost_model", d["cost_model"])
print("config3", json.dumps(d.get("config3"))[:1500])
print("config5", json.dumps(d.get("config5"))[:400])
print("config4", [(r["bytes"], r["algo"], r["flexar_busbw"], r["correct"]) for r in d.get("config4", {}).get("rows", [])])
PY
tail -5 gpurun_out/r6_n8/rehearse_rccl_n8.log | cut -c1-600
exit $rc
