#!/bin/bash
# Large-message executor efficiency on one GPU (ranks share the HBM): per-kernel times under rocprofv3.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/probe_large" -o run -- python3 "$R/bench/protocol_probe.py" --manifest "$R/gpurun_out/probe_large_manifest.json" --ranks 2,8 --kib 16384,65536 --specs "flat+pull,flat+push,flat+pull+wt,flat+push+wt,flat+pull+nts,ring,ring+wt,oneshot" --grids "32,64,128" --reps 5 > "$R/gpurun_out/probe_large.log" 2>&1 ) && \
python3 bench/protocol_probe.py --parse gpurun_out/probe_large/run_kernel_trace.csv --manifest gpurun_out/probe_large_manifest.json > gpurun_out/probe_large.jsonl && echo "probe ok"
