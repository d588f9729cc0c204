#!/bin/bash
# Round 5: the same counters as gpu_r5o.sh for the fp8 reduction after the packed converters (final tree).
# one rocprofv3 pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass), each pass bounded with
# SIGKILL at 90 s; then one kernel trace of the same cases for the times.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5t
export FLEXAR_NO_BUILD=1
O="$R/gpurun_out/r5t"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
for dt in float8_e4m3fn; do
  for k in 2 8; do
    for grp in FETCH_SIZE WRITE_SIZE SQ; do
      ctr="$grp"; [ $grp = SQ ] && ctr="$SQ"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv \
          -d "$O/${dt}_k${k}_$grp" -o run -- python3 "$R/bench/kernel_bench.py" --what reduce --dtypes $dt --fanins $k \
          --iters 5 > "$O/${dt}_k${k}_$grp.log" 2>&1) || { echo "pmc $dt k$k $grp failed"; exit 1; }
    done
    echo "pmc $dt k$k ok"
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- \
    python3 "$R/bench/kernel_bench.py" --what reduce --dtypes float8_e4m3fn --fanins 2,8 --iters 5 > "$O/trace.log" 2>&1) && echo "trace ok" || exit 1
python3 bench/reduce_pmc_summary.py gpurun_out/r5t
