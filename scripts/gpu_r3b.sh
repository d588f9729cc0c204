#!/bin/bash
# Round 3, second GPU pass: the driver's N>1 bench flow with every BASELINE config section, RCCL in the loop
# (one NCCL_HOSTID per rank on the shared GPU), N = 2 and N = 4, default arguments (budget 400 s); then the
# N = 1 bench under rocprofv3 kernel stats. Each step has its own time limit; steps chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/r3_rehearse_n2.log 2>&1 && echo "rehearse n=2 ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 560 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 10 --warmup 3 \
    > gpurun_out/r3_rehearse_n4.log 2>&1 && echo "rehearse n=4 ok"
rc=$?
grep '^{' gpurun_out/r3_rehearse_n2.log > gpurun_out/r3_bench_shared_n2.json 2>/dev/null
grep '^{' gpurun_out/r3_rehearse_n4.log > gpurun_out/r3_bench_shared_n4.json 2>/dev/null
python3 - <<'PY' 2>/dev/null
import json
for n in (2, 4):
    try:
        d = json.load(open(f"gpurun_out/r3_bench_shared_n{n}.json"))
    except Exception as e:
        print(n, "no line", e); continue
    print(n, "value", d["value"], "alg", d["config"]["algorithm"], "wall", d["bench_wall_s"], "dropped", d["dropped"])
    print("  cost_model", d["cost_model"])
    print("  calib", {k: d["readiness"]["calibration"].get(k) for k in ("source", "alpha_launch_us", "alpha_sync_us", "link_gbps", "hbm_gbps", "median_rel_err", "ms")})
    print("  config3", json.dumps(d.get("config3"))[:600])
    print("  config5", json.dumps(d.get("config5"))[:400])
    print("  config4", [(r["bytes"], r["algo"], r["flexar_busbw"], r.get("rccl_busbw"), r["correct"]) for r in d.get("config4", {}).get("rows", [])])
PY
exit $rc
