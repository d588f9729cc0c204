#!/bin/bash
# Per-kernel protocol cost sweep (ranks x size x algorithm x grid) on one GPU under rocprofv3.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/probe" -o run -- python3 "$R/bench/protocol_probe.py" --manifest "$R/gpurun_out/probe_manifest.json" "$@" > "$R/gpurun_out/probe.log" 2>&1 ) && \
python3 bench/protocol_probe.py --parse gpurun_out/probe/run_kernel_trace.csv --manifest gpurun_out/probe_manifest.json > gpurun_out/probe.jsonl && echo "probe ok"
