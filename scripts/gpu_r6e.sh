#!/bin/bash
# Round 6, fifth pass: (1) rhd vs rhd:7 on the in-process group kernel at the SAME workgroups per rank (28: a
# multiple of 7), to separate the channels' own cost from the grid rounding to whole channels; (2) the LL /
# small-message latency floor with the crash report's progress stores on (default) and off
# (FLEXAR_CRASH_REPORT=0), 2 processes on one GPU, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6e
export FLEXAR_NO_BUILD=1
out=gpurun_out/r6e/channels_grid28.jsonl
: > $out
for rep in 1 2; do
  for spec in "rhd+pull" "tree:2,2,2:7+pull" "tree:4,2+pull" "tree:4,2:7+pull"; do
    line=$(TEP_GRID=28 TEP_RANKS=8 TEP_MIB=64 timeout -k 10 120 python3 bench/typed_exec_probe.py "$spec" float32 \
           2>>gpurun_out/r6e/err.log | grep '^{') || { echo "probe $spec failed"; exit 1; }
    echo "{\"grid_per_rank\": 28, \"rep\": $rep, ${line:1}" | tee -a $out
  done
done
for rep in 1 2; do
  for cr in 1 0; do
    FLEXAR_CRASH_REPORT=$cr timeout -k 10 200 python3 bench/latency_ipc.py --nranks 2 --iters 400 --algos ll,oneshot \
        --sizes 8,256,4096,65536 --out gpurun_out/r6e/lat_cr${cr}_rep$rep.jsonl > gpurun_out/r6e/lat_cr${cr}_rep$rep.log 2>&1 ||
        { echo "latency cr=$cr failed"; exit 1; }
  done
done
echo "latency ok"
for f in gpurun_out/r6e/lat_*.jsonl; do echo "== $f"; cat $f; done
