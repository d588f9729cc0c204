#!/bin/bash
# Round 3: the program-cost model against FETCH/WRITE_SIZE, then the typed-executor efficiency probe.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
bash scripts/gpu_pmc_model.sh > /dev/null && echo "pmc ok" && bash scripts/gpu_typed_probe.sh
rc=$?
cat gpurun_out/pmc_model/summary.txt 2>/dev/null
exit $rc
