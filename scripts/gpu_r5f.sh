#!/bin/bash
# Round 5: the grid-interleaved standalone reduction, grid cap x per-lane unroll at high fan-in (the default build,
# U = 1 for fan-in 5-8, against a FLEXAR_UNROLL_WIDE=2 build), fan-in 2 / 4 / 8, 256 MiB per source, 2 reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5f
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5f
for rep in 1 2; do
  for v in b1024 b512 b256 w1024 w512; do
    case $v in b*) L=allreduce_over_mpi_amd/_lib/libflexar.so;; w*) L=allreduce_over_mpi_amd/_lib_u2w/libflexar.so;; esac
    FLEXAR_LIB_PATH="$R/$L" FLEXAR_REDUCE_GRID=${v:1} timeout -k 10 120 python3 bench/kernel_bench.py --what reduce \
        --fanins 2,4,8 --iters 20 > $O/$v.$rep.jsonl 2> $O/$v.$rep.err || { echo "$v failed"; exit 1; }
    echo "$v.$rep ok"
  done
done
python3 - <<'PY'
import glob, json, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r5f/*.jsonl")):
    v = f.split("/")[-1].split(".")[0]
    for line in open(f):
        d = json.loads(line)
        rows[(d["dtype"], d["fanin"], v)].append(d["eff_TBps"])
for k in sorted(rows):
    print(k, [round(x, 3) for x in rows[k]])
PY
