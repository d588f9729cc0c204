#!/bin/bash
# Round 4: HBM bytes of the MX executor (FETCH_SIZE and WRITE_SIZE in runs of their own: 3 + 2 TCC counters
# exceed one run's 4) against the program model. SIGKILL-bounded passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/mx_bytes
export FLEXAR_NO_BUILD=1 TEP_ITERS=5
for c in FETCH_SIZE WRITE_SIZE; do
  for spec in flat+pull+mxe4m3 fp8; do
    tag="${c}_$(echo $spec | tr '+' '_')"
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv \
        -d "$R/gpurun_out/mx_bytes/$tag" -o run -- python3 "$R/bench/typed_exec_probe.py" $spec bfloat16 \
        > "$R/gpurun_out/mx_bytes/$tag.log" 2>&1) || { echo "pmc $tag failed"; exit 1; }
    echo "pmc $tag ok"
  done
done
