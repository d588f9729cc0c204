#!/bin/bash
# Round 5: the executor with two 16-B groups in flight for fan-in 5-8 XFERs (FLEXAR_UNROLL_WIDE=2 build) against the
# default, in-process groups of 2 / 4 / 8 ranks (bench/kernel_bench.py --what group), libraries interleaved, 2 reps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5g
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5g
for rep in 1 2; do
  for v in base u2w; do
    case $v in base) L=allreduce_over_mpi_amd/_lib/libflexar.so;; u2w) L=allreduce_over_mpi_amd/_lib_u2w/libflexar.so;; esac
    FLEXAR_LIB_PATH="$R/$L" timeout -k 10 200 python3 bench/kernel_bench.py --what group > $O/$v.$rep.jsonl 2> $O/$v.$rep.err \
        || { echo "$v failed"; exit 1; }
    echo "$v.$rep ok"
  done
done
python3 - <<'PY'
import glob, json, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r5g/*.jsonl")):
    v = f.split("/")[-1].split(".")[0]
    for line in open(f):
        d = json.loads(line)
        if "us" in d and d["KiB"] >= 16384:
            rows[(d["nranks"], d["KiB"], d["algo"], v)].append(d["us"])
for k in sorted(rows):
    print(k, rows[k])
PY
