#!/bin/bash
# Round 6, third pass: the MX codec on non-finite input (NaN sign byte fix), then the typed-executor workgroup A/B
#  on the in-process group kernel (one launch holds every rank: co-residency is the launch's
# own): bench/typed_exec_probe.py, 4 ranks x 100 MiB, shipped 512-thread build vs abv/ (FLEXAR_TYPED_THREADS=256,
# grid x2-3 capped by residency), interleaved A B A B; then rocprofv3 kernel traces of one probe per build.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6c
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_mx.py > gpurun_out/r6c/mx.log 2>&1 && echo "mx ok" || exit 1
out=gpurun_out/r6c/typed_ab.jsonl
: > $out
for rep in 1 2; do
  for c in "flat+pull float32" "fp8 bfloat16" "fp8 float32" "flat+pull+mxe4m3 float32" "flat+pull+mxe4m3 bfloat16" "rhd+pull+f32 bfloat16"; do
    set -- $c
    for lib in base t256; do
      if [ "$lib" = t256 ]; then export FLEXAR_LIB_PATH="$R/abv/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
      line=$(timeout -k 10 120 python3 bench/typed_exec_probe.py "$1" "$2" 2>>gpurun_out/r6c/err.log | grep '^{') ||
        { echo "probe $c ($lib) failed"; exit 1; }
      echo "{\"build\": \"$lib\", \"rep\": $rep, ${line:1}" | tee -a $out
    done
  done
done
for lib in base t256; do
  if [ "$lib" = t256 ]; then export FLEXAR_LIB_PATH="$R/abv/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c/prof_$lib -o run -- python3 bench/typed_exec_probe.py fp8 bfloat16 \
      > gpurun_out/r6c/prof_$lib.log 2>&1 || { echo "prof $lib failed"; exit 1; }
done
unset FLEXAR_LIB_PATH
echo "ab done"
