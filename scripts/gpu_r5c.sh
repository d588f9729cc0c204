#!/bin/bash
# Round 5: (1) the MX codec after the wave-contiguous pack (bitwise tests, probe); (2) the readiness tests that
# changed; (3) the 8-process self-launched shared-GPU rehearsal of bench.py ONCE, with the
# per-rank phase logs and the crash report on, its whole stderr kept. Each GPU step bounded, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5c
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5c
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mx.py -x -v -m gpu -k codec --timeout 240 --timeout-method thread \
    > $O/tests_codec.log 2>&1 && echo "codec tests ok" &&
timeout -k 10 200 python3 bench/hier_mx_probe.py > $O/hier_mx_probe.jsonl 2> $O/hier_mx_probe.err && echo "codec probe ok" &&
cat $O/hier_mx_probe.jsonl &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bench.py tests/test_gpu_ipc.py -x -v -m gpu -k "recovered or readiness_gate" \
    --timeout 240 --timeout-method thread > $O/tests_readiness.log 2>&1 && echo "readiness tests ok" &&
FLEXAR_BENCH_SHARED_GPU=1 FLEXAR_BENCH_SHARED_RCCL=1 timeout -k 10 500 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
    > $O/bench_selflaunch_n8.json 2> $O/bench_selflaunch_n8.err && echo "n=8 ok"
rc=$?
tail -3 $O/tests_readiness.log 2>/dev/null
python3 -c "import json; d=json.load(open('$O/bench_selflaunch_n8.json')); print(d['value'], d.get('bench_wall_s'), json.dumps(d.get('readiness',{}).get('selftest_recovered')), json.dumps(d.get('config5')))" 2>/dev/null
exit $rc
