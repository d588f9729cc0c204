#!/bin/bash
# Round 4: typed executors run the last, partial super-group lane-interleaved too (range-checked buffer descriptors; the contiguous layout only for write-through) - after the full-super-group change (not only multiples
# of UU). Correctness (typed / fp8 / MX tests, 2- and 4-rank matrices) then timings at DDP bucket size
# (25 MiB) and at 100 MiB for the fp8 wires and the fp32-partials schedules.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4t
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4t
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mx.py tests/test_gpu_kernels.py -x -v -k "mx or fp8 or typed or f32 or partials or misaligned" \
    --timeout 240 --timeout-method thread > $O/tests_typed.log 2>&1 && echo "typed tests ok" &&
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_multidevice.py -x -v -k "acceptance_matrix and (n2 or n4)" --timeout 450 \
    --timeout-method thread > $O/test_gpu_multidevice.log 2>&1 && echo "multidevice ok" || exit 1
: > $O/timings.jsonl
for mib in 1 25 100; do
  for c in "fp8 float32" "flat+pull+mxe4m3 float32" "fp8 bfloat16" "flat+pull+mxe4m3 bfloat16" "rhd+pull+f32 bfloat16" "ring+f32 bfloat16" "flat+pull float32"; do
    set -- $c
    TEP_MIB=$mib TEP_ITERS=20 timeout -k 10 120 python3 bench/typed_exec_probe.py $1 $2 >> $O/timings.jsonl || exit 1
  done
done
cat $O/timings.jsonl
