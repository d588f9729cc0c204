#!/bin/bash
# Round 5, combined first pass (GPU slots are scarce): r5a (new GPU tests, N = 1 bench with reduce_kernel, its
# kernel-trace profile), the MX codec probe, then the typed-executor batch-depth A/B (r5b, one repetition,
# base library measured before and after the variants). Each GPU step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5a gpurun_out/r5b
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5a
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lifecycle.py tests/test_gpu_bench.py tests/test_gpu_mx.py -x -v -m gpu \
    --timeout 240 --timeout-method thread > $O/tests.log 2>&1 && echo "tests ok" &&
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err && echo "profile ok" &&
timeout -k 10 200 python3 bench/hier_mx_probe.py > $O/hier_mx_probe.jsonl 2> $O/hier_mx_probe.err && echo "codec probe ok" &&
cat $O/hier_mx_probe.jsonl || { rc=$?; tail -5 $O/tests.log; exit $rc; }
B=gpurun_out/r5b
export TEP_ITERS=20 TEP_MIB=100 TEP_RANKS=4
for lib in base uuA uuB base2; do
  case $lib in base|base2) L=allreduce_over_mpi_amd/_lib/libflexar.so;; *) L=allreduce_over_mpi_amd/_lib_$lib/libflexar.so;; esac
  for c in "fp8 bfloat16" "fp8 float32" "flat+pull+mxe4m3 float32" "flat+pull+mxe4m3 bfloat16" "flat+pull float32"; do
    set -- $c
    tag="$(echo $1 | tr '+' '_')_$2"
    FLEXAR_LIB_PATH="$R/$L" timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $B/$lib/$tag.1 -o run -- \
        python3 bench/typed_exec_probe.py $1 $2 >> $B/$lib.jsonl 2>> $B/$lib.err || { echo "$lib $tag failed"; exit 1; }
  done
  echo "$lib ok"
done
python3 bench/kstats_summary.py $B > $B/summary.txt && cat $B/summary.txt
