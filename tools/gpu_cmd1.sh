# ad-hoc GPU batch of the session
set -o pipefail
mkdir -p gpurun_out/r5m
timeout -k 10 600 python -u -m pytest tests/test_gpu_topology.py tests/test_gpu_assume.py tests/test_gpu_static_plugins.py -v --timeout 300 --timeout-method thread > gpurun_out/r5m/topo.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/r5m/topo.log | head -30; exit 1; }
tail -2 gpurun_out/r5m/topo.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5m/prof -o c2t -- python3 bench.py --config c2d --no-c5 --no-sub --no-cpu-baseline --no-profile --steps 1 --warmup 0 --pods 2000 > gpurun_out/r5m/prof_bench.json 2> gpurun_out/r5m/prof_bench.err || { tail -20 gpurun_out/r5m/prof_bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c2d --no-c5 --no-sub --steps 2 --warmup 1 --detail gpurun_out/r5m/c2t_detail.json > gpurun_out/r5m/c2t.json 2> gpurun_out/r5m/c2t.err || { tail -20 gpurun_out/r5m/c2t.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/r5m/c2t.json
