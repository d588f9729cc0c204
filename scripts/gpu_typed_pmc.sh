#!/bin/bash
# Where the typed (fp8-wire) executor spends its wave cycles next to the untyped flat: one rocprofv3 --pmc pass
# of 8 SQ counters per case over bench/typed_exec_probe.py (4 ranks in one launch, 100 MiB per rank). Each pass
# is its own bounded run (SIGKILL at 90 s: a counter request the hardware cannot hold hangs instead of failing).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/typed_pmc
export FLEXAR_NO_BUILD=1 TEP_ITERS=5
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/typed_pmc/counters.txt" 2>&1) || true
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for c in "flat+pull float32" "fp8 float32" "fp8 bfloat16"; do
  set -- $c
  tag="$1_$2"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv \
      -d "$R/gpurun_out/typed_pmc/$tag" -o run -- python3 "$R/bench/typed_exec_probe.py" "$1" "$2" \
      > "$R/gpurun_out/typed_pmc/$tag.log" 2>&1) || { echo "pmc $tag failed"; exit 1; }
  echo "pmc $tag ok"
done
