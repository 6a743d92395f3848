set -o pipefail
mkdir -p gpurun_out/pre1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c3_policy.py tests/test_gpu_numa_policy.py tests/test_gpu_deviceshare.py tests/test_gpu_deviceshare_joint.py tests/test_gpu_numa.py tests/test_gpu_cpuset.py tests/test_gpu_cpu_bind.py tests/test_gpu_parity.py tests/test_gpu_shard_loopback.py > gpurun_out/pre1/pytest.log 2>&1 &&
KS_PRE_RSV=0 timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-c5 --no-preempt > gpurun_out/pre1/c3_off.json 2>gpurun_out/pre1/c3_off.err &&
timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-c5 --no-preempt > gpurun_out/pre1/c3_on.json 2>gpurun_out/pre1/c3_on.err &&
timeout -k 10 200 python tools/diag_commit.py c3 > gpurun_out/pre1/diag_c3.log 2>&1
