#!/bin/bash
# fp8-compressed allreduce: fused (round 2) vs launch chain (round 1) vs plain; kernel trace for launch
# counts and per-kernel time; FETCH_SIZE / WRITE_SIZE of one fused call vs one chain.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/fp8
export FLEXAR_NO_BUILD=1
timeout -k 10 300 python3 bench/fp8_allreduce_bench.py > gpurun_out/fp8/bench.jsonl 2> gpurun_out/fp8/bench.err && echo "bench ok" &&
(cd /tmp && export TMPDIR=/tmp && FP8B_MIB=25 FP8B_ITERS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/fp8/trace" -o run -- python3 "$R/bench/fp8_allreduce_bench.py" > "$R/gpurun_out/fp8/trace.log" 2>&1) && echo "trace ok" &&
(cd /tmp && export TMPDIR=/tmp && FP8B_MIB=25 FP8B_ITERS=5 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d "$R/gpurun_out/fp8/pmc" -o run -- python3 "$R/bench/fp8_allreduce_bench.py" > "$R/gpurun_out/fp8/pmc.log" 2>&1) && echo "pmc fetch ok" &&
(cd /tmp && export TMPDIR=/tmp && FP8B_MIB=25 FP8B_ITERS=5 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv \
    -d "$R/gpurun_out/fp8/pmcw" -o run -- python3 "$R/bench/fp8_allreduce_bench.py" > "$R/gpurun_out/fp8/pmcw.log" 2>&1) && echo "pmc write ok"
rc=$?
cat gpurun_out/fp8/bench.jsonl
exit $rc
