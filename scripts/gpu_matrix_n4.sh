set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
export FLEXAR_NO_BUILD=1
timeout -k 10 600 python3 -u -m pytest "tests/test_gpu_multidevice.py::test_acceptance_matrix[n4-shared-gpu0]" -x -v -s --timeout 500 --timeout-method thread > gpurun_out/matrix_n4.log 2>&1
rc=$?
grep -n "rank\|PASS\|FAIL\|Error" gpurun_out/matrix_n4.log | tail -40
exit $rc
