#!/bin/bash
# Round 5: (1) exec_body's XFER split back to one call site, so the transfer is inlined again (two call sites had
# made the compiler outline it into a called function with a stack frame); (2) the typed executors' software
# pipelining A/B (FLEXAR_TYPED_PIPE_MAXV=16 build in _lib_pipe: batch i+1's loads issued before batch i's stores);
# (3) the chunked work split re-measured without the outlined call. Correctness first, then 2 reps of
# base / pipe / base+chunks: untyped schedules in one launch (kernel_bench group) and the typed executors under
# rocprofv3 (typed_exec_probe, 4 ranks x 100 MiB).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r5j
export FLEXAR_NO_BUILD=1 TMPDIR=/tmp
O=gpurun_out/r5j
PIPE="$R/allreduce_over_mpi_amd/_lib_pipe/libflexar.so"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu --timeout 240 --timeout-method thread \
    > $O/tests_base.log 2>&1 && echo "base kernel tests ok" && tail -1 $O/tests_base.log || { tail -30 $O/tests_base.log; exit 1; }
FLEXAR_LIB_PATH="$PIPE" timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q -m gpu \
    --timeout 240 --timeout-method thread > $O/tests_pipe.log 2>&1 && echo "pipe kernel tests ok" && tail -1 $O/tests_pipe.log \
    || { tail -30 $O/tests_pipe.log; exit 1; }
export TEP_ITERS=20 TEP_MIB=100 TEP_RANKS=4
for rep in 1 2; do
  for cfg in base pipe chunk; do
    L=""; I=0
    case $cfg in pipe) L="$PIPE";; chunk) I=1;; esac
    FLEXAR_LIB_PATH="$L" FLEXAR_EXEC_INTERLEAVE=$I timeout -k 10 200 python3 bench/kernel_bench.py --what group \
        > $O/group_$cfg.$rep.jsonl 2> $O/group_$cfg.$rep.err || { echo "group $cfg failed"; exit 1; }
    for c in "fp8 bfloat16" "fp8 float32" "flat+pull+mxe4m3 float32" "flat+pull+mxe4m3 bfloat16" "flat+pull float32"; do
      set -- $c
      tag="$(echo $1 | tr '+' '_')_$2"
      FLEXAR_LIB_PATH="$L" FLEXAR_EXEC_INTERLEAVE=$I timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$cfg/$tag.$rep -o run -- \
          python3 bench/typed_exec_probe.py $1 $2 >> $O/typed_$cfg.jsonl 2>> $O/typed_$cfg.err || { echo "$cfg $tag failed"; exit 1; }
    done
    echo "rep $rep $cfg ok"
  done
done
python3 bench/kstats_summary.py $O | grep -v "^$"
python3 - <<'PY'
import glob, json, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r5j/group_*.jsonl")):
    v = f.split("/")[-1].split(".")[0]
    for line in open(f):
        d = json.loads(line)
        if "us" in d and d["KiB"] >= 1024:
            rows[(d["nranks"], d["KiB"], d["algo"], v)].append(d["us"])
for k in sorted(rows):
    print(k, rows[k])
PY
