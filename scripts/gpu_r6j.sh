#!/bin/bash
# Round 6: progress words only for launches >= 1 MiB - the GPU test of the report, then the small-call latency
# with the report on (default) and off, interleaved, 3 reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6j
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_crash_progress.py \
    tests/test_crash_report.py > gpurun_out/r6j/test.log 2>&1 && echo "tests ok" || { tail -30 gpurun_out/r6j/test.log; exit 1; }
for rep in 1 2 3; do
  for mode in on off; do
    case $mode in on) e="";; off) e="FLEXAR_CRASH_REPORT=0";; esac
    env $e timeout -k 10 200 python3 bench/latency_ipc.py --nranks 2 --iters 400 --algos ll,oneshot \
        --sizes 8,4096,65536 --out gpurun_out/r6j/lat_${mode}_rep$rep.jsonl > gpurun_out/r6j/lat_${mode}_rep$rep.log 2>&1 ||
        { echo "latency $mode failed"; exit 1; }
  done
done
python3 - <<'PY'
import glob, json, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r6j/lat_*.jsonl"):
    mode = f.split("lat_")[1].split("_rep")[0]
    for l in open(f):
        d = json.loads(l)
        if d["algo"] in ("ll", "oneshot"):
            agg[(d["algo"], d["bytes"], mode)].append(d["us_per_call"])
for k in sorted(agg):
    v = agg[k]
    print(k, round(sum(v) / len(v), 2), v)
PY
