#!/bin/bash
# Round 5: packed fp8 arithmetic in combine16 (v1 = this tree; v2 = the same plus 4 waves per SIMD on the
# reduction, FLEXAR_REDUCE_OCC4=1; v0 = the previous commit, per-element converts). Kernel tests with each
# library (the new saturation / NaN test included), then the standalone reduction, two reps, libraries interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5p
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5p
lib() { case $1 in v1) echo "";; v2) echo "$R/allreduce_over_mpi_amd/_lib_occ4/libflexar.so";; v0) echo "$R/allreduce_over_mpi_amd/_lib_v0/libflexar.so";; esac; }
for v in v1 v2 v0; do
  FLEXAR_LIB_PATH="$(lib $v)" timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu \
      --timeout 240 --timeout-method thread > $O/tests_$v.log 2>&1 && echo "$v kernel tests ok" && tail -1 $O/tests_$v.log \
      || { tail -30 $O/tests_$v.log; exit 1; }
done
for rep in 1 2; do
  for v in v0 v1 v2; do
    FLEXAR_LIB_PATH="$(lib $v)" timeout -k 10 300 python3 bench/kernel_bench.py --what reduce --fanins 1,2,4,8 \
        > $O/reduce_$v.$rep.jsonl 2> $O/reduce_$v.$rep.err || { echo "reduce $v failed"; exit 1; }
    echo "rep $rep $v ok"
  done
done
python3 - <<'PY'
import glob, json, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r5p/reduce_*.jsonl")):
    v = f.split("/")[-1].split(".")[0].split("_")[1]
    for line in open(f):
        d = json.loads(line)
        rows[(d["dtype"], d["fanin"], v)].append(d["eff_TBps"])
for k in sorted(rows):
    print(k, rows[k])
PY
