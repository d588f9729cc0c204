#!/bin/bash
# Round 5, typed-executor batch depth A/B: the default library against builds with deeper
# per-lane load batches (FLEXAR_TYPED_UU2_MAXV / UU4_MAXV), 4 ranks in one launch, 100 MiB per rank, every case
# under rocprofv3 --kernel-trace --stats (per-kernel device time), libraries interleaved, two repetitions.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5b
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp TEP_ITERS=20 TEP_MIB=100 TEP_RANKS=4
O=gpurun_out/r5b
for rep in 1 2; do
  for lib in base uuA uuB; do
    case $lib in base) L=allreduce_over_mpi_amd/_lib/libflexar.so;; *) L=allreduce_over_mpi_amd/_lib_$lib/libflexar.so;; esac
    [ -f "$L" ] || continue
    for c in "fp8 bfloat16" "fp8 float32" "flat+pull+mxe4m3 float32" "flat+pull+mxe4m3 bfloat16" "flat+pull float32"; do
      set -- $c
      tag="$(echo $1 | tr '+' '_')_$2"
      FLEXAR_LIB_PATH="$R/$L" timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$lib/$tag.$rep -o run -- \
          python3 bench/typed_exec_probe.py $1 $2 >> $O/$lib.jsonl 2>> $O/$lib.err || { echo "$lib $tag failed"; exit 1; }
    done
    echo "rep $rep $lib ok"
  done
done
python3 bench/kstats_summary.py $O > $O/summary.txt && cat $O/summary.txt
