#!/bin/bash
# Round 4, A/B: the MX executor with every fan-in (the library) vs one built for fan-ins <= 4 only
# (-DFLEXAR_MXB_KMAX4, abk4/): does the K 5..8 code's register pressure cost the 4-rank kernel?
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4k
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r4k
: > $O/ab.jsonl
for rep in 1 2; do
  for lib in main k4; do
    for dt in bfloat16 float32; do
      if [ $lib = k4 ]; then export FLEXAR_LIB_PATH=$R/abk4/libflexar.so; else unset FLEXAR_LIB_PATH; fi
      echo -n "{\"lib\": \"$lib\", \"r\": " >> $O/ab.jsonl
      timeout -k 10 120 python3 bench/typed_exec_probe.py flat+pull+mxe4m3 $dt >> $O/ab.jsonl || exit 1
      sed -i '$ s/$/}/' $O/ab.jsonl
    done
  done
done
cat $O/ab.jsonl
