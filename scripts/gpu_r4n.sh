#!/bin/bash
# Round 4: SQ counters of the MX executor next to the global-scale fp8 executor and the untyped flat (bf16
# and fp32 inputs, 4 ranks in one launch, 100 MiB per rank), plus one HBM-bytes pass (FETCH_SIZE /
# WRITE_SIZE) of the MX kernel against the program model. One bounded pmc pass per run (SIGKILL at 90 s).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/mx_pmc
export FLEXAR_NO_BUILD=1 TEP_ITERS=5
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for c in "flat+pull+mxe4m3 bfloat16" "fp8 bfloat16" "flat+pull+mxe4m3 float32" "fp8 float32" "flat+pull float32"; do
  set -- $c
  tag="$(echo $1 | tr '+' '_')_$2"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv \
      -d "$R/gpurun_out/mx_pmc/$tag" -o run -- python3 "$R/bench/typed_exec_probe.py" "$1" "$2" \
      > "$R/gpurun_out/mx_pmc/$tag.log" 2>&1) || { echo "pmc $tag failed"; exit 1; }
  echo "pmc $tag ok"
done
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv \
    -d "$R/gpurun_out/mx_pmc/bytes_mx_bf16" -o run -- python3 "$R/bench/typed_exec_probe.py" flat+pull+mxe4m3 bfloat16 \
    > "$R/gpurun_out/mx_pmc/bytes_mx_bf16.log" 2>&1) || { echo "pmc bytes failed"; exit 1; }
echo "pmc bytes ok"
python3 bench/pmc_sq_summary.py gpurun_out/mx_pmc > gpurun_out/mx_pmc/sq_counters.txt 2>&1
cat gpurun_out/mx_pmc/sq_counters.txt
