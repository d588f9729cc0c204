#!/bin/bash
# BASELINE.json configs #3-#5 through the driver's bench flow, rehearsed with 4 ranks on ONE GPU
# (FLEXAR_BENCH_SHARED_GPU=1: shared HBM, gloo reference; not xGMI numbers):
#   #3 RHD bf16 1 GiB (forced rhd+pull, and the tuner's own choice)
#   #4 buffer sweep 4 KiB -> 1 GiB with the cost-model/tune-table selection
#   #5 fp8 e4m3 gradient allreduce with the fused 1/N post-scale (op avg)
# Each step bounded; chained with && so the first failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/configs
export FLEXAR_NO_BUILD=1 FLEXAR_BENCH_SHARED_GPU=1
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
      --master-port 29610 bench.py --gpus 4 "$@" > gpurun_out/configs/$name.log 2>&1 && echo "$name ok"
}
run c3_rhd_bf16_1g --dtype bfloat16 --size-mb 1024 --algo rhd+pull --steps 5 --warmup 2 &&
run c3_auto_bf16_1g --dtype bfloat16 --size-mb 1024 --steps 5 --warmup 2 &&
run c5_fp8_avg --dtype float8_e4m3fn --op avg --steps 10 --warmup 3 &&
run c4_sweep --size-mb 4 --no-tune --steps 5 --warmup 2 --sweep 4K:1G --sweep-out gpurun_out/configs/sweep.jsonl
rc=$?
for f in gpurun_out/configs/*.log; do echo "== $f"; tail -1 "$f" | cut -c1-400; done
exit $rc
