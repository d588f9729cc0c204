#!/bin/bash
# Round 5: the standalone reduction, per-workgroup slices against the grid-interleaved form (and its grid cap),
# fan-in 1..8, fp32 / bf16 / fp8, 256 MiB per source; then the reduce GPU tests on the default. Bounded, &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5e
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5e
for rep in 1 2; do
  for v in slices inter inter512 inter2048; do
    case $v in
      slices) E="FLEXAR_REDUCE_SLICES=1";; inter) E="";; inter512) E="FLEXAR_REDUCE_GRID=512";; inter2048) E="FLEXAR_REDUCE_GRID=2048";;
    esac
    env $E timeout -k 10 120 python3 bench/kernel_bench.py --what reduce --fanins 2,4,8 --iters 20 > $O/$v.$rep.jsonl 2> $O/$v.$rep.err \
        || { echo "$v failed"; exit 1; }
    echo "$v.$rep ok"
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "reduce" --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
    && echo "reduce tests ok" && tail -2 $O/tests.log
rc=$?
python3 - <<'PY'
import glob, json, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r5e/*.jsonl")):
    v = f.split("/")[-1].split(".")[0]
    for line in open(f):
        d = json.loads(line)
        rows[(d["dtype"], d["fanin"], v)].append(d["eff_TBps"])
for k in sorted(rows):
    print(k, [round(x, 3) for x in rows[k]])
PY
exit $rc
