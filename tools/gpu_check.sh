#!/bin/bash
# One GPU call: parity tests, smoke(), bench (with CPU baseline), rocprofv3 kernel stats.
set -o pipefail
OUT=gpurun_out/${1:-run}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -30 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
