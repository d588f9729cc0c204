#!/bin/bash
# Round 6, second pass: MPI zero copy by default, the shared-GPU acceptance matrix (channelled trees included),
# the N=1 bench, then the typed-executor workgroup A/B: 512-thread (shipped) vs the
# 256-thread build in abv/ (FLEXAR_TYPED_THREADS=256), one process per rank on one GPU, interleaved A B A B,
# with per-kernel VGPR / occupancy of both builds. Each GPU step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6b
export FLEXAR_NO_BUILD=1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_mpi.py > gpurun_out/r6b/mpi.log 2>&1 && echo "mpi ok" &&
timeout -k 10 900 $PYT tests/test_gpu_multidevice.py > gpurun_out/r6b/multidevice.log 2>&1 && echo "multidevice ok" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6b/bench_n1.log 2>&1 && echo "bench ok" || exit 1
# MX codec on non-finite input: a plain test failure (rc 1) is data, anything else ends the call
timeout -k 10 300 $PYT tests/test_gpu_mx.py -k codec > gpurun_out/r6b/mx_codec.log 2>&1
mrc=$?; echo "mx codec rc=$mrc"; [ $mrc -le 1 ] || exit $mrc
for lib in base t256; do
  if [ "$lib" = t256 ]; then export FLEXAR_LIB_PATH="$R/abv/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
  timeout -k 10 120 python bench/kernel_info.py > gpurun_out/r6b/kinfo_$lib.txt 2>&1 || { echo "kinfo $lib failed"; exit 1; }
done &&
unset FLEXAR_LIB_PATH &&
for rep in 1 2; do
  for lib in base t256; do
    if [ "$lib" = t256 ]; then export FLEXAR_LIB_PATH="$R/abv/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
    timeout -k 10 240 python bench/typed_mp_probe.py flat:float32 fp8:bfloat16 fp8:float32 mx:float32 mx:bfloat16 \
        2>>gpurun_out/r6b/probe_err.log | sed "s/^{/{\"build\": \"$lib\", \"rep\": $rep, /" >> gpurun_out/r6b/typed_mp.jsonl ||
        { echo "probe $lib failed"; exit 1; }
  done
done && echo "typed A/B ok"
rc=$?
unset FLEXAR_LIB_PATH
for f in gpurun_out/r6b/*.log; do echo "== $f"; tail -3 "$f" | cut -c1-300; done
cat gpurun_out/r6b/typed_mp.jsonl 2>/dev/null
exit $rc
