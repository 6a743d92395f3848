set -o pipefail
mkdir -p gpurun_out/q4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_assume.py tests/test_gpu_shard_loopback.py tests/test_gpu_static_plugins.py > gpurun_out/q4/pytest.log 2>&1 &&
for i in 1 2; do timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sub --no-c5 --no-preempt >> gpurun_out/q4/c2.json 2>>gpurun_out/q4/c2.err || exit 1; done
