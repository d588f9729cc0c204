#!/bin/bash
# Round 4: 8-rank fp8 wires after the register cut of the masked partial super-group (MX KMAX 8 no longer
# spills): one launch of 8 ranks (100 MiB fp32 per rank), then the self-launched 8-rank bench rehearsal.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4u
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4u
: > $O/n8.jsonl
for spec in fp8 flat+pull+mxe4m3 flat+pull; do
  TEP_RANKS=8 TEP_MIB=100 TEP_ITERS=10 timeout -k 10 180 python3 bench/typed_exec_probe.py $spec float32 >> $O/n8.jsonl || exit 1
done
cat $O/n8.jsonl
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n8.json 2> $O/bench_selflaunch_n8.err && echo "n=8 ok"
rc=$?
python3 -c "import json; d=json.load(open('$O/bench_selflaunch_n8.json')); print(d['value'], json.dumps(d.get('config5')), d.get('bench_wall_s'))"
exit $rc
