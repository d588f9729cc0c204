#!/bin/bash
# Round 4, eleventh GPU pass: fp8-wire kernels in two fan-in classes (KMAX 4 / 8). Correctness first (MX and
# global-scale fp8 group tests, the 2- and 4-rank multi-process matrices), then the 4-rank, 100 MiB timings
# of both fp8 wires against the untyped flat, and a kernel trace of each fp8 form.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4l
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r4l
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mx.py tests/test_gpu_kernels.py -x -v -k "mx or fp8 or typed or f32 or partials" \
    --timeout 240 --timeout-method thread > $O/tests_fp8_mx.log 2>&1 && echo "fp8/mx tests ok" &&
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_multidevice.py -x -v -k "acceptance_matrix and (n2 or n4)" --timeout 450 \
    --timeout-method thread > $O/test_gpu_multidevice.log 2>&1 && echo "multidevice ok" || exit 1
: > $O/mx_ab.jsonl
for rep in 1 2; do
  for dt in bfloat16 float32; do
    for spec in fp8 flat+pull+mxe4m3 flat+pull; do
      timeout -k 10 120 python3 bench/typed_exec_probe.py $spec $dt >> $O/mx_ab.jsonl || exit 1
    done
  done
done
cat $O/mx_ab.jsonl
for spec in fp8 flat+pull+mxe4m3; do
  tag=$(echo $spec | tr '+' '_')
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python3 bench/typed_exec_probe.py $spec bfloat16 \
      > $O/prof_$tag.json 2>&1 || exit 1
done
echo profiles ok
