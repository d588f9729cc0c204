#!/bin/bash
# Round 4, fifth GPU pass: the driver's N > 1 bench flow through bench.py's own launcher (no torchrun), N = 2,
# 4 and 8 ranks on one GPU with RCCL (every config section, wall time), then one rocprofv3 SQ-counter pass per
# typed-executor case (scripts/gpu_typed_pmc.sh's counters) on the round-4 build. Each GPU step bounded.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4e/typed_pmc
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4e
for n in 2 4 8; do
  FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus $n --steps 10 --warmup 3 \
      > $O/bench_selflaunch_n$n.json 2> $O/bench_selflaunch_n$n.err || { echo "self-launch n=$n failed"; tail -20 $O/bench_selflaunch_n$n.err; exit 1; }
  echo "self-launch n=$n ok"
done
export TEP_ITERS=5
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for c in "flat+pull float32" "fp8 float32" "fp8 bfloat16" "rhd+pull+f32 bfloat16" "rhd+pull+rw bfloat16"; do
  set -- $c
  tag="$1_$2"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv \
      -d "$R/$O/typed_pmc/$tag" -o run -- python3 "$R/bench/typed_exec_probe.py" "$1" "$2" \
      > "$R/$O/typed_pmc/$tag.log" 2>&1) || { echo "pmc $tag failed"; exit 1; }
  echo "pmc $tag ok"
done
python3 bench/pmc_sq_summary.py $O/typed_pmc > $O/typed_pmc/sq_counters.txt && cat $O/typed_pmc/sq_counters.txt
