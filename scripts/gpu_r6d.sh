#!/bin/bash
# Round 6, fourth pass (shared-HBM rehearsals, not xGMI numbers):
#  1. flexar_bench (the reference CLI, MPI_Allreduce_FT path) on 4 ranks sharing the GPU, 64 MiB fp32: staging
#     (FLEXAR_MPI_ZC=0) vs the new default (registration + zero copy), schedule and time per size;
#  2. multi-channel trees vs single-channel on the in-process group kernel (8 ranks x 64 MiB): flat, rhd, rhd:7,
#     tree:4,2, tree:4,2:7 (fp32) and rhd / rhd:7 with fp32 partials (bf16): on one HBM the channels cannot win
#     links, this prices their overhead;
#  3. rocprofv3 kernel trace of the rhd:7 group run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r6d
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
MPIRUN=/opt/conda/bin/mpirun
for mode in staging zc; do
  if [ $mode = staging ]; then export FLEXAR_MPI_ZC=0; else unset FLEXAR_MPI_ZC; fi
  FLEXAR_MAX_GRID=16 FLEXAR_TIMEOUT_MS=20000 timeout -k 10 240 $MPIRUN -np 4 bin/flexar_bench --mem device \
      --sweep 4M:64M --repeat 20 --warmup 5 > gpurun_out/r6d/fbench_$mode.log 2>&1 || { echo "flexar_bench $mode failed"; exit 1; }
  echo "flexar_bench $mode ok"
done
unset FLEXAR_MPI_ZC
out=gpurun_out/r6d/channels.jsonl
: > $out
for c in "flat+pull float32" "rhd+pull float32" "tree:2,2,2:7+pull float32" "tree:4,2+pull float32" "tree:4,2:7+pull float32" \
         "rhd+push float32" "tree:2,2,2:7+push float32" "rhd+pull+f32 bfloat16" "tree:2,2,2:7+pull+f32 bfloat16"; do
  set -- $c
  TEP_RANKS=8 TEP_MIB=64 timeout -k 10 120 python3 bench/typed_exec_probe.py "$1" "$2" 2>>gpurun_out/r6d/err.log | grep '^{' >> $out ||
      { echo "probe $c failed"; exit 1; }
done
echo "channels ok"
TEP_RANKS=8 TEP_MIB=64 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d/prof_rhd7 -o run -- \
    python3 bench/typed_exec_probe.py "tree:2,2,2:7+pull" float32 > gpurun_out/r6d/prof_rhd7.log 2>&1 || { echo "prof failed"; exit 1; }
TEP_RANKS=8 TEP_MIB=64 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d/prof_rhd -o run -- \
    python3 bench/typed_exec_probe.py "rhd+pull" float32 > gpurun_out/r6d/prof_rhd.log 2>&1 || { echo "prof failed"; exit 1; }
echo "prof ok"
cat $out
grep -E "^ +[0-9]+ " gpurun_out/r6d/fbench_*.log
grep -h "schedule" gpurun_out/r6d/fbench_*.log | sort | uniq -c
