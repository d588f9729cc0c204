#!/bin/bash
# Zero-copy vs staging flat: timing lines and a rocprofv3 kernel-stats run of the same script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 bench/zc_bench.py > gpurun_out/zc_bench.jsonl 2> gpurun_out/zc_bench.err && echo "zc bench ok" &&
(cd /tmp && export TMPDIR=/tmp && ZCB_RANKS=2,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_zc" -o run -- python3 "$R/bench/zc_bench.py" > "$R/gpurun_out/prof_zc.log" 2>&1) && echo "prof ok"
rc=$?
cat gpurun_out/zc_bench.jsonl
exit $rc
