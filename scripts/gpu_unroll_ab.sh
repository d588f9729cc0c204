#!/bin/bash
# A/B of the high-fan-in unroll (FLEXAR_UNROLL_WIDE 1 vs 2): executor occupancy / VGPRs, the LocalGroup
# zero-copy and staging flat schedules, and the standalone reduce kernel at fan-in 8.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/ab
export FLEXAR_NO_BUILD=1
V=allreduce_over_mpi_amd/_lib/variants/libflexar_u2.so
timeout -k 10 120 python3 bench/kernel_info.py > gpurun_out/ab/info_u1.jsonl 2>&1 &&
FLEXAR_LIB_PATH=$R/$V timeout -k 10 120 python3 bench/kernel_info.py > gpurun_out/ab/info_u2.jsonl 2>&1 &&
ZCB_RANKS=4,8 timeout -k 10 200 python3 bench/zc_bench.py > gpurun_out/ab/zc_u1.jsonl 2>gpurun_out/ab/zc_u1.err &&
FLEXAR_LIB_PATH=$R/$V ZCB_RANKS=4,8 timeout -k 10 200 python3 bench/zc_bench.py > gpurun_out/ab/zc_u2.jsonl 2>gpurun_out/ab/zc_u2.err &&
echo "ab ok"
timeout -k 10 200 python3 bench/kernel_bench.py --what reduce --fanins 5,8 --dtypes float32,bfloat16 > gpurun_out/ab/red_u1.jsonl 2>&1 &&
FLEXAR_LIB_PATH=$R/$V timeout -k 10 200 python3 bench/kernel_bench.py --what reduce --fanins 5,8 --dtypes float32,bfloat16 > gpurun_out/ab/red_u2.jsonl 2>&1 &&
echo "reduce ab ok"
