#!/bin/bash
# the whole -m gpu suite, then the default bench line without c5 (c2 + c3 / c4 / c2d / preempt records)
set -o pipefail
OUT=gpurun_out/${1:-q}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --no-c5 ${BENCH_ARGS:---no-cpu-baseline} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json
