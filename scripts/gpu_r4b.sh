#!/bin/bash
# Round 4, second GPU pass:
#  0. the c10d backend GPU tests (host-page agreements for the zero-copy probe);
#  1. bench.py's own launcher: `bench.py --gpus N` with no torchrun, N = 2 and 4 ranks on one GPU (RCCL flow);
#  2. the fan-in-2 executor instantiations A/B (FLEXAR_KMAX_SPECIALIZE 1 vs 0, interleaved, two reps):
#     bench/typed_exec_probe.py, 4 ranks in one launch, 100 MiB per rank;
#  3. the DDP step A/B (c10d backend default / without zero copy / hook / RCCL) at 2 and 4 ranks.
# Each GPU step bounded; steps chained with && (the first failure ends the call).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4b
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4b
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_backend.py -x -v --timeout 240 --timeout-method thread \
    > $O/test_gpu_backend.log 2>&1 && echo "backend tests ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n2.json 2> $O/bench_selflaunch_n2.err && echo "self-launch n=2 ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 400 python3 bench.py --gpus 4 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n4.json 2> $O/bench_selflaunch_n4.err && echo "self-launch n=4 ok" || exit 1
out=$O/kmax_ab.jsonl
: > "$out"
for rep in 1 2; do
  for c in "rhd+pull+f32 bfloat16" "rhd+pull+rw bfloat16" "ring+f32 bfloat16" "fp8 bfloat16" "flat+pull float32" "ring float32" "rhd float32"; do
    set -- $c
    for k in 1 0; do
      line=$(FLEXAR_KMAX_SPECIALIZE=$k timeout -k 10 120 python3 bench/typed_exec_probe.py "$1" "$2" 2>>$O/kmax_err.log | grep '^{') ||
        { echo "probe $c (kmax=$k) failed"; exit 1; }
      echo "{\"kmax_specialize\": $k, \"rep\": $rep, ${line:1}" | tee -a "$out"
    done
  done
done
DDPB_RANKS=2 timeout -k 10 400 python3 bench/ddp_step_bench.py > $O/ddp_n2.jsonl 2> $O/ddp_n2.err && echo "ddp n=2 ok" &&
DDPB_RANKS=4 timeout -k 10 500 python3 bench/ddp_step_bench.py > $O/ddp_n4.jsonl 2> $O/ddp_n4.err && echo "ddp n=4 ok"
rc=$?
cat $O/ddp_n2.jsonl $O/ddp_n4.jsonl 2>/dev/null
exit $rc
