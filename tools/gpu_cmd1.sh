set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 400 python -u -m pytest tests/test_gpu_preempt.py tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5a/new.log 2>&1 || { tail -50 gpurun_out/r5a/new.log; exit 1; }
tail -3 gpurun_out/r5a/new.log
BENCH=1 BENCH_ARGS="--steps 10 --warmup 3" bash tools/gpu_tests.sh r5a
