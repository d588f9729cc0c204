#!/bin/bash
# A/B: 8-bit PROD / MAX / MIN transfers with one 16-B group per lane (abv/byteu1, FLEXAR_BYTE_OP_U1=1) against the
# shipped unroll; 4 ranks x 64 MiB in one launch, builds alternated, 2 repetitions, results checked exactly.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6y
export FLEXAR_NO_BUILD=1
for rep in 1 2; do
  for lib in base u1; do
    if [ $lib = u1 ]; then export FLEXAR_LIB_PATH="$R/abv/byteu1/libflexar.so"; else unset FLEXAR_LIB_PATH; fi
    timeout -k 10 240 python3 bench/byte_op_probe.py 2>>gpurun_out/r6y/err.log | grep '^{' >> gpurun_out/r6y/time.jsonl ||
        { echo "probe $lib failed"; exit 1; }
  done
done
unset FLEXAR_LIB_PATH
python3 - <<'PY' | tee gpurun_out/r6y/summary.txt
import json
rows = {}
bad = 0
for l in open("gpurun_out/r6y/time.jsonl"):
    d = json.loads(l)
    bad += not d["exact"]
    rows.setdefault((d["spec"], d["dtype"], d["op"]), {}).setdefault(d["lib"] or "_lib", []).append(d["us_per_call"])
print("inexact results:", bad)
for k, v in sorted(rows.items()):
    print(k, {lib: sorted(x) for lib, x in v.items()})
PY
