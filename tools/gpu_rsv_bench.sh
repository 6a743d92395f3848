#!/bin/bash
# Reservation parity tests then the C4 bench (no CPU baseline).
set -o pipefail
OUT=gpurun_out/${1:-rb}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_reservation.py -x -q --timeout 180 --timeout-method thread > $OUT/pytest_rsv.log 2>&1 || { echo "rsv pytest failed"; tail -60 $OUT/pytest_rsv.log; exit 1; }
tail -2 $OUT/pytest_rsv.log
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
