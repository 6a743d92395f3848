#!/bin/bash
# GPU parity tests (optionally a subset: $2 = pytest -k expression, or TESTS="file ..."), then smoke(), then (BENCH=1)
# the default bench line without c5 (BENCH_ARGS to change it).
set -o pipefail
OUT=gpurun_out/${1:-t}
mkdir -p $OUT
timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread ${2:+-k} ${2:+"$2"} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---no-c5 --no-cpu-baseline} --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
  python3 tools/bench_summary.py $OUT/bench.json
fi
