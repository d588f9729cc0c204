#!/bin/bash
# Every Python example, briefly, with 2 ranks sharing one GPU (gloo fallback group, co-resident grids): DDP over
# the "flexar" backend / the hook / the zero-copy hook / the fp8 hook / RCCL, FSDP2, MoE all-to-all, and the
# tensor-parallel decode step (eager vs hipGraph). Each run bounded; the first failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/examples
export FLEXAR_NO_BUILD=1 FLEXAR_PG_FALLBACK=gloo FLEXAR_MAX_GRID=16
run() {  # name, then the torchrun arguments
  local name=$1; shift
  timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29600 + RANDOM % 300)) "$@" > "gpurun_out/examples/$name.log" 2>&1 || { echo "$name FAILED"; return 1; }
  echo "$name ok: $(grep '^{' "gpurun_out/examples/$name.log" | tail -1 | cut -c1-400)"
}
for c in backend hook zchook fp8hook; do
  run "ddp_$c" examples/train_ddp.py --comm "$c" --model gpt-tiny --steps 5 --warmup 2 --bucket-mb auto || exit 1
done
run fsdp examples/train_fsdp.py --model gpt-tiny --steps 5 --warmup 2 || exit 1
run moe examples/moe_dispatch.py || exit 1
run moe_zc examples/moe_dispatch.py --zero-copy || exit 1
timeout -k 10 240 python3 examples/tp_decode.py --nranks 2 --layers 8 --steps 20 > gpurun_out/examples/tp_decode.log 2>&1 \
    && echo "tp_decode ok: $(tail -3 gpurun_out/examples/tp_decode.log | cut -c1-400)" || { echo "tp_decode FAILED"; exit 1; }
