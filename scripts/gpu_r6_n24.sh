#!/bin/bash
# The driver's N = 2 and N = 4 bench runs, rehearsed on a 1-GPU box (ranks share device 0, RCCL over loopback
# sockets), on the final tree. Each step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6_n24
export FLEXAR_NO_BUILD=1 FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 GPU_MAX_HW_QUEUES=2
for n in 2 4; do
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 10 --warmup 3 \
      > gpurun_out/r6_n24/rehearse_n$n.log 2>&1 || { echo "n=$n failed"; exit 1; }
  grep '^{' gpurun_out/r6_n24/rehearse_n$n.log > gpurun_out/r6_n24/bench_shared_n$n.json
  python3 - "$n" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r6_n24/bench_shared_n{sys.argv[1]}.json"))
bad = [k for k, v in d.items() if isinstance(v, dict) and v.get("correct") is False]
print("n", sys.argv[1], "value", d["value"], "alg", d["config"]["algorithm"], "wall", d["bench_wall_s"],
      "dropped", d["dropped"], "incorrect sections", bad)
print("config4", [(r["bytes"], r["algo"], r["correct"]) for r in d.get("config4", {}).get("rows", [])])
PY
done
