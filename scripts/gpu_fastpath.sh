set -o pipefail
export FLEXAR_NO_BUILD=1 FLEXAR_TIMEOUT_MS=10000
mkdir -p gpurun_out
OUT=lat_eager2.jsonl bash scripts/gpu_latency.sh > gpurun_out/lat_a.txt 2>&1 && echo lat_ok &&
timeout -k 10 120 python bench/latency_ipc.py --nranks 2 --graph --algos oneshot,flat --sizes 256,4,8,16,64,4 --out gpurun_out/lat_probe.jsonl > gpurun_out/lat_b.txt 2>&1 && echo probe_ok &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ipc.py tests/test_gpu_faults.py tests/test_gpu_backend.py > gpurun_out/pytest_fast.txt 2>&1; rc=$?; tail -5 gpurun_out/pytest_fast.txt; exit $rc
