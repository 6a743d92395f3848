mkdir -p gpurun_out/f4 && timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f4/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/f4/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-c5 --no-cpu-baseline > gpurun_out/f4/bench.json 2> gpurun_out/f4/bench.err || exit 1
python3 tools/bench_summary.py gpurun_out/f4/bench.json
