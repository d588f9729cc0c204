#!/bin/bash
# Round 4, seventh GPU pass: the fp8 wire on gfx950's scaled converts (power-of-two pre-scale; push,
# all-gather and own contributions in one conversion per element pair): the fp8 GPU tests, an A/B of the
# typed probe against ab/libflexar.so (the library before the change), and one SQ-counter pass per fp8 case.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4g/typed_pmc
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4g
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -v -k "fp8 or typed or partials" --timeout 240 \
    --timeout-method thread > $O/test_fp8.log 2>&1 && echo "fp8 kernel tests ok" || { tail -40 $O/test_fp8.log; exit 1; }
out=$O/fp8_ab.jsonl
: > "$out"
for rep in 1 2; do
  for c in "fp8 bfloat16" "fp8 float32" "flat+pull float32" "fp8 float16"; do
    set -- $c
    for lib in new base; do
      if [ "$lib" = base ]; then export FLEXAR_LIB_PATH="$R/ab/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
      line=$(timeout -k 10 120 python3 bench/typed_exec_probe.py "$1" "$2" 2>>$O/ab_err.log | grep '^{') ||
        { echo "probe $c ($lib) failed"; exit 1; }
      echo "{\"lib\": \"$lib\", \"rep\": $rep, ${line:1}" | tee -a "$out"
    done
  done
done
unset FLEXAR_LIB_PATH
export TEP_ITERS=5
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for c in "flat+pull float32" "fp8 float32" "fp8 bfloat16"; do
  set -- $c
  tag="$1_$2"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv \
      -d "$R/$O/typed_pmc/$tag" -o run -- python3 "$R/bench/typed_exec_probe.py" "$1" "$2" \
      > "$R/$O/typed_pmc/$tag.log" 2>&1) || { echo "pmc $tag failed"; exit 1; }
  echo "pmc $tag ok"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$O/kstats_fp8_bf16" -o run -- python3 "$R/bench/typed_exec_probe.py" fp8 bfloat16 > "$R/$O/kstats.log" 2>&1) &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$O/kstats_flat_f32" -o run -- python3 "$R/bench/typed_exec_probe.py" flat+pull float32 >> "$R/$O/kstats.log" 2>&1) &&
python3 bench/pmc_sq_summary.py $O/typed_pmc > $O/typed_pmc/sq_counters.txt && cat $O/typed_pmc/sq_counters.txt
