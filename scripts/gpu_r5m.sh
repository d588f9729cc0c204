#!/bin/bash
# Round 5: untyped paths in the typed kernels capped (fp8 wire: copies only; validator matches), and the narrow
# global-scale fp8 kernels at 3 waves per SIMD (FLEXAR_TYPED_OCC3=1 build in _lib_occ3). Kernel tests with both
# libraries, then the typed probe (4 ranks x 100 MiB in one launch) under rocprofv3, 2 reps, libraries interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5m
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5m
OCC="$R/allreduce_over_mpi_amd/_lib_occ3/libflexar.so"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu --timeout 240 --timeout-method thread \
    > $O/tests_base.log 2>&1 && echo "base kernel tests ok" && tail -1 $O/tests_base.log || { tail -30 $O/tests_base.log; exit 1; }
FLEXAR_LIB_PATH="$OCC" timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu \
    --timeout 240 --timeout-method thread > $O/tests_occ3.log 2>&1 && echo "occ3 kernel tests ok" && tail -1 $O/tests_occ3.log \
    || { tail -30 $O/tests_occ3.log; exit 1; }
export TEP_ITERS=20 TEP_MIB=100 TEP_RANKS=4
for rep in 1 2; do
  for cfg in base occ3; do
    L=""; [ $cfg = occ3 ] && L="$OCC"
    for c in "fp8 bfloat16" "fp8 float32" "flat+pull+mxe4m3 float32" "flat+pull float32"; do
      set -- $c
      tag="$(echo $1 | tr '+' '_')_$2"
      FLEXAR_LIB_PATH="$L" timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$cfg/$tag.$rep -o run -- \
          python3 bench/typed_exec_probe.py $1 $2 >> $O/typed_$cfg.jsonl 2>> $O/typed_$cfg.err || { echo "$cfg $tag failed"; exit 1; }
    done
    echo "rep $rep $cfg ok"
  done
done
python3 bench/kstats_summary.py $O | grep -v "^$"
