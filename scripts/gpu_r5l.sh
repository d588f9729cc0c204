#!/bin/bash
# Round 5, final tree: the driver's round-end order (whole GPU tier, smoke(), N = 1 bench), a kernel trace of the
# bench, then one rocprofv3 --pmc pass of 8 SQ counters per typed case (4 ranks x 100 MiB in one launch; each pass
# bounded with SIGKILL at 90 s). Every step bounded, chained.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5l
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5l
timeout -k 10 1000 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > $O/test_gpu_all.log 2>&1 && echo "gpu tests ok" && tail -1 $O/test_gpu_all.log || { tail -30 $O/test_gpu_all.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n=1 ok" && cat $O/bench_n1.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
    > $O/bench_n1_prof.json 2> $O/bench_n1_prof.err && echo "profile ok" || exit 1
export TEP_ITERS=5
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for c in "flat+pull float32" "fp8 bfloat16" "flat+pull+mxe4m3 float32"; do
  set -- $c
  tag="$(echo $1 | tr '+' '_')_$2"
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv \
      -d "$R/$O/pmc/$tag" -o run -- python3 "$R/bench/typed_exec_probe.py" "$1" "$2" \
      > "$R/$O/pmc_$tag.log" 2>&1) || { echo "pmc $tag failed"; exit 1; }
  echo "pmc $tag ok"
done
python3 bench/pmc_sq_summary.py $O/pmc
