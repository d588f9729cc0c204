#!/bin/bash
# Round 3, third GPU pass: the N = 1 bench and its rocprofv3 kernel stats, then the program-cost model
# against FETCH_SIZE / WRITE_SIZE (scripts/gpu_pmc_model.sh). Steps chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 bench.py > gpurun_out/r3_bench_n1.log 2>&1 && echo "bench n=1 ok" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/r3_prof_bench" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 \
    > "$R/gpurun_out/r3_prof_bench.log" 2>&1) && echo "prof ok" &&
bash scripts/gpu_pmc_model.sh
rc=$?
tail -1 gpurun_out/r3_bench_n1.log | cut -c1-400
exit $rc
