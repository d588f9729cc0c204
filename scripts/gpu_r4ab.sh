#!/bin/bash
# Round 4, the OCP MX wire incl. the reduce-scatter - the group tests (bit for bit against the
# reference arithmetic), the fp8 / typed kernel tests (the scaled-convert helpers now take per-run scales),
# and the 2-rank multi-process matrix (exec kernel). Each GPU step bounded; chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out/r4ab
export FLEXAR_NO_BUILD=1
O=gpurun_out/r4ab
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mx.py -x -v --timeout 240 --timeout-method thread \
    > $O/test_gpu_mx.log 2>&1 && echo "mx group tests ok" &&
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -v -k "fp8 or typed or f32 or partials" --timeout 240 --timeout-method thread \
    > $O/test_gpu_kernels_fp8.log 2>&1 && echo "fp8/typed kernel tests ok" &&
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_multidevice.py -x -v -k "acceptance_matrix and (n2 or n4)" --timeout 450 --timeout-method thread \
    > $O/test_gpu_multidevice.log 2>&1 && echo "multidevice ok"
rc=$?
for f in $O/*.log; do echo "== $f"; tail -4 $f; done
exit $rc
