#!/bin/bash
# Round 6: where the crash report's small-call cost goes - breadcrumbs + device progress stores (default), the
# breadcrumbs alone (FLEXAR_PROGRESS=0) and neither (FLEXAR_CRASH_REPORT=0); 2 processes on one GPU, LL and
# oneshot, interleaved, 3 reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6i
export FLEXAR_NO_BUILD=1
for rep in 1 2 3; do
  for mode in on noprog off; do
    case $mode in on) e="";; noprog) e="FLEXAR_PROGRESS=0";; off) e="FLEXAR_CRASH_REPORT=0";; esac
    env $e timeout -k 10 200 python3 bench/latency_ipc.py --nranks 2 --iters 400 --algos ll,oneshot \
        --sizes 8,4096 --out gpurun_out/r6i/lat_${mode}_rep$rep.jsonl > gpurun_out/r6i/lat_${mode}_rep$rep.log 2>&1 ||
        { echo "latency $mode failed"; exit 1; }
  done
done
python3 - <<'PY'
import glob, json, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r6i/lat_*.jsonl"):
    mode = f.split("lat_")[1].split("_rep")[0]
    for l in open(f):
        d = json.loads(l)
        if d["algo"] in ("ll", "oneshot"):
            agg[(d["algo"], d["bytes"], mode)].append(d["us_per_call"])
for k in sorted(agg):
    v = agg[k]
    print(k, round(sum(v) / len(v), 2), v)
PY
