set -o pipefail
mkdir -p gpurun_out/q5
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c3_policy.py tests/test_gpu_numa_policy.py tests/test_gpu_deviceshare.py tests/test_gpu_static_plugins.py tests/test_gpu_balanced.py tests/test_gpu_reservation.py tests/test_gpu_assume.py > gpurun_out/q5/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-c5 --no-cpu-baseline --no-preempt > gpurun_out/q5/bench.json 2> gpurun_out/q5/bench.err && python3 tools/bench_summary.py gpurun_out/q5/bench.json
