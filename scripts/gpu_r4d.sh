#!/bin/bash
# Round 4, fourth GPU pass:
#  1. the GPU tests touched by the partials default ("auto") and the misaligned path: test_gpu_kernels.py and
#     the acceptance matrix (test_gpu_multidevice.py);
#  2. A/B of the unconditional post-scale (no per-element select) and the partials forms: the library under
#     test vs ab/libflexar_base.so (FLEXAR_LIB_PATH), bench/typed_exec_probe.py, 4 ranks in one launch,
#     100 MiB per rank, interleaved, two reps;
#  3. the 4-rank DDP hook case with variants (2 hardware queues per process; staging instead of zero copy;
#     "+nts") to find what costs it 100 ms per step.
# Each GPU step bounded; chained with && (the first failure ends the call).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4d
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4d
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multidevice.py -x -v --timeout 240 \
    --timeout-method thread > $O/test_kernels_matrix.log 2>&1 && echo "kernel + matrix tests ok" || { tail -30 $O/test_kernels_matrix.log; exit 1; }
out=$O/scale_ab.jsonl
: > "$out"
for rep in 1 2; do
  for c in "rhd+pull+f32 bfloat16" "rhd+pull+rw bfloat16" "rhd+pull bfloat16" "ring+f32 bfloat16" "fp8 bfloat16" "fp8 float32" "flat+pull float32" "rhd float32"; do
    set -- $c
    for lib in new base; do
      if [ "$lib" = base ]; then export FLEXAR_LIB_PATH="$R/ab/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
      line=$(timeout -k 10 120 python3 bench/typed_exec_probe.py "$1" "$2" 2>>$O/scale_err.log | grep '^{') ||
        { echo "probe $c ($lib) failed"; exit 1; }
      echo "{\"lib\": \"$lib\", \"rep\": $rep, ${line:1}" | tee -a "$out"
    done
  done
done
unset FLEXAR_LIB_PATH
DDPB_RANKS=4 DDPB_MODES=hook DDPB_STEP_SYNC=1 GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python3 bench/ddp_step_bench.py \
    > $O/ddp_hook_q2.jsonl 2> $O/ddp_hook_q2.err && echo "hook q2 ok" &&
DDPB_RANKS=4 DDPB_MODES=hook DDPB_STEP_SYNC=1 FLEXAR_HOOK_ZC=0 timeout -k 10 200 python3 bench/ddp_step_bench.py \
    > $O/ddp_hook_nozc.jsonl 2> $O/ddp_hook_nozc.err && echo "hook nozc ok" &&
DDPB_RANKS=4 DDPB_MODES=hook DDPB_STEP_SYNC=1 DDPB_HOOK_ALGO=flat+nts timeout -k 10 200 python3 bench/ddp_step_bench.py \
    > $O/ddp_hook_nts.jsonl 2> $O/ddp_hook_nts.err && echo "hook nts ok"
rc=$?
grep -h '^{' $O/ddp_hook_*.jsonl
exit $rc
