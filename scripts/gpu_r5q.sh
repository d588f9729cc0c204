#!/bin/bash
# Round 5: the adopted packed fp8 arithmetic (fence kernels; 4 waves per SIMD on the fp8 reduction; write-through
# kernels keep per-element converts) against v0 (the commit before it): kernel tests, the standalone reduction,
# and the untyped fp8 executor (flat+pull on fp8 tensors, 4 ranks x 100 MiB in one launch, under rocprofv3).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5q
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5q
V0="$R/allreduce_over_mpi_amd/_lib_v0/libflexar.so"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu --timeout 240 --timeout-method thread \
    > $O/tests_new.log 2>&1 && echo "kernel tests ok" && tail -1 $O/tests_new.log || { tail -30 $O/tests_new.log; exit 1; }
export TEP_ITERS=20 TEP_MIB=100 TEP_RANKS=4
for rep in 1 2; do
  for v in v0 new; do
    L=""; [ $v = v0 ] && L="$V0"
    FLEXAR_LIB_PATH="$L" timeout -k 10 300 python3 bench/kernel_bench.py --what reduce --dtypes float8_e4m3fn,float8_e5m2,float32 \
        --fanins 2,4,8 > $O/reduce_$v.$rep.jsonl 2> $O/reduce_$v.$rep.err || { echo "reduce $v failed"; exit 1; }
    FLEXAR_LIB_PATH="$L" timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$v/flat_pull_fp8.$rep -o run -- \
        python3 bench/typed_exec_probe.py flat+pull float8_e4m3fn >> $O/typed_$v.jsonl 2>> $O/typed_$v.err || { echo "exec $v failed"; exit 1; }
    echo "rep $rep $v ok"
  done
done
python3 bench/kstats_summary.py $O | grep -v "^$"
python3 - <<'PY'
import glob, json, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r5q/reduce_*.jsonl")):
    v = f.split("/")[-1].split(".")[0].split("_")[1]
    for line in open(f):
        d = json.loads(line)
        rows[(d["dtype"], d["fanin"], v)].append(d["eff_TBps"])
for k in sorted(rows):
    print(k, rows[k])
PY
