#!/bin/bash
# Round 4, third GPU pass: the DDP step A/B again after closing the zero-copy probe window early
# (FLEXAR_PG_ZC_IDLE_STOP) with per-step diagnostics of the 4-rank hook case, the backend GPU tests, the
# N=1 bench and its rocprofv3 kernel stats. Each GPU step bounded; chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4c
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4c
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_backend.py -x -v --timeout 240 --timeout-method thread \
    > $O/test_gpu_backend.log 2>&1 && echo "backend tests ok" &&
DDPB_RANKS=4 DDPB_MODES=hook,hook,pg DDPB_STEP_SYNC=1 timeout -k 10 400 python3 bench/ddp_step_bench.py \
    > $O/ddp_n4_diag.jsonl 2> $O/ddp_n4_diag.err && echo "ddp n=4 diag ok" &&
DDPB_RANKS=2 DDPB_MODES=pg,pg_nozc,hook timeout -k 10 400 python3 bench/ddp_step_bench.py > $O/ddp_n2.jsonl 2> $O/ddp_n2.err &&
DDPB_RANKS=4 DDPB_MODES=pg,pg_nozc timeout -k 10 400 python3 bench/ddp_step_bench.py > $O/ddp_n4.jsonl 2> $O/ddp_n4.err &&
echo "ddp ok" &&
timeout -k 10 300 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo "bench n1 ok" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_bench" \
    -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$R/$O/prof_bench.log" 2>&1) && echo "prof ok"
rc=$?
cat $O/ddp_n4_diag.jsonl $O/ddp_n2.jsonl $O/ddp_n4.jsonl 2>/dev/null | grep '^{'
exit $rc
