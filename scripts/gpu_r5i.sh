#!/bin/bash
# Round 5: executor XFER work split - per-workgroup slices (default) against round-robin kXferChunk chunks
# (FLEXAR_EXEC_INTERLEAVE=1): correctness first (the group / typed kernel tests with the chunks), then untyped
# schedules in one launch (kernel_bench group) and the typed executors under rocprofv3 (typed_exec_probe), 2 reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5i
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5i
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu -k chunked --timeout 240 --timeout-method thread \
    > $O/tests_chunked.log 2>&1 && echo "chunked split exact" && tail -1 $O/tests_chunked.log || { tail -30 $O/tests_chunked.log; exit 1; }
FLEXAR_EXEC_INTERLEAVE=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu \
    --timeout 240 --timeout-method thread > $O/tests_interleave.log 2>&1 && echo "tests with chunks ok" && tail -1 $O/tests_interleave.log \
    || { tail -30 $O/tests_interleave.log; exit 1; }
export TEP_ITERS=20 TEP_MIB=100 TEP_RANKS=4
for rep in 1 2; do
  for v in 0 1; do
    FLEXAR_EXEC_INTERLEAVE=$v timeout -k 10 200 python3 bench/kernel_bench.py --what group > $O/group_i$v.$rep.jsonl 2> $O/group_i$v.$rep.err \
        || { echo "group i$v failed"; exit 1; }
    for c in "fp8 bfloat16" "flat+pull+mxe4m3 float32" "flat+pull float32" "fp8 float32"; do
      set -- $c
      tag="$(echo $1 | tr '+' '_')_$2"
      FLEXAR_EXEC_INTERLEAVE=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/i$v/$tag.$rep -o run -- \
          python3 bench/typed_exec_probe.py $1 $2 >> $O/typed_i$v.jsonl 2>> $O/typed_i$v.err || { echo "i$v $tag failed"; exit 1; }
    done
    echo "rep $rep i$v ok"
  done
done
python3 bench/kstats_summary.py $O | grep -v "^$" 
python3 - <<'PY'
import glob, json, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r5i/group_*.jsonl")):
    v = f.split("/")[-1].split(".")[0]
    for line in open(f):
        d = json.loads(line)
        if "us" in d and d["KiB"] >= 1024:
            rows[(d["nranks"], d["KiB"], d["algo"], v)].append(d["us"])
for k in sorted(rows):
    print(k, rows[k])
PY
