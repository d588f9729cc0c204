#!/bin/bash
# Round 6: per-process executors read their by-value context through the kernarg segment (no scratch). Small-call
# latency, 2 processes on one GPU, the same runs as gpu_r6i.sh (crash report on) for comparison, 3 reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6t
export FLEXAR_NO_BUILD=1
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench/latency_ipc.py --nranks 2 --iters 400 --algos ll,oneshot,flat \
      --sizes 8,4096,65536,1048576 --out gpurun_out/r6t/lat_rep$rep.jsonl > gpurun_out/r6t/lat_rep$rep.log 2>&1 ||
      { echo "latency rep $rep failed"; exit 1; }
done
python3 - <<'PY' | tee gpurun_out/r6t/summary.txt
import glob, json, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6t/lat_rep*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        agg[(d["algo"], d["bytes"])].append(d["us_per_call"])
for k in sorted(agg):
    print(k, sorted(agg[k]))
PY
