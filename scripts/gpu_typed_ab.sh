#!/bin/bash
# A/B of the typed executor on one box: bench/typed_exec_probe.py (4 ranks in one launch, 100 MiB per rank,
# hipEvent-timed, model HBM bytes) for each case with the library under test and with the baseline build in
# ab/libflexar_base.so (FLEXAR_LIB_PATH), interleaved A B A B so box drift hits both. Each run bounded.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/typed_ab
export FLEXAR_NO_BUILD=1
out=gpurun_out/typed_ab/summary.jsonl
: > "$out"
for rep in 1 2; do
  for c in "fp8 float32" "fp8 bfloat16" "rhd+pull+f32 bfloat16" "ring+f32 bfloat16" "flat+pull float32"; do
    set -- $c
    for lib in new base; do
      if [ "$lib" = base ]; then export FLEXAR_LIB_PATH="$R/ab/libflexar_base.so"; else unset FLEXAR_LIB_PATH; fi
      line=$(timeout -k 10 120 python3 bench/typed_exec_probe.py "$1" "$2" 2>>gpurun_out/typed_ab/err.log | grep '^{') ||
        { echo "probe $c ($lib) failed"; exit 1; }
      echo "{\"lib\": \"$lib\", \"rep\": $rep, ${line:1}" | tee -a "$out"
    done
  done
done
unset FLEXAR_LIB_PATH
