#!/bin/bash
# Round 5: the driver's round-end order on the current tree (whole GPU tier, smoke(), N = 1 bench), then the MX
# executor's scale-byte gather A/B: the default (one 1-B scale access per wave and operand, cross-lane reads)
# against _lib_nogather (one 1-B access per lane, run and operand), 4 and 8 ranks in one launch x 100 MiB,
# under rocprofv3 --kernel-trace --stats, two repetitions. Every step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5k
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5k
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/test_gpu_all.log 2>&1 && echo "gpu tests ok" && tail -1 $O/test_gpu_all.log || { tail -30 $O/test_gpu_all.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json || exit 1
NG="$R/allreduce_over_mpi_amd/_lib_nogather/libflexar.so"
FLEXAR_LIB_PATH="$NG" timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mx.py -x -q -m gpu --timeout 240 --timeout-method thread \
    > $O/tests_nogather.log 2>&1 && echo "nogather mx tests ok" || { tail -30 $O/tests_nogather.log; exit 1; }
export TEP_ITERS=20 TEP_MIB=100
for rep in 1 2; do
  for lib in base nogather; do
    L=""; [ $lib = nogather ] && L="$NG"
    for nr in 4 8; do
      for dt in float32 bfloat16; do
        FLEXAR_LIB_PATH="$L" TEP_RANKS=$nr timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$lib/mx_n${nr}_$dt.$rep -o run -- \
            python3 bench/typed_exec_probe.py flat+pull+mxe4m3 $dt >> $O/typed_$lib.jsonl 2>> $O/typed_$lib.err \
            || { echo "$lib n$nr $dt failed"; exit 1; }
      done
    done
    echo "rep $rep $lib ok"
  done
done
python3 bench/kstats_summary.py $O | grep -v "^$"
