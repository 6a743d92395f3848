#!/bin/bash
# Quick GPU iteration: parity tests, commit-phase diagnostics, short C2 bench.
set -o pipefail
OUT=gpurun_out/${1:-q}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
if [ -f koordinator_amd/libkoordgpu_diag.so ]; then
  timeout -k 10 120 python -u tools/diag_commit.py > $OUT/diag.txt 2>&1 || { echo "diag failed"; tail -20 $OUT/diag.txt; exit 1; }
  cat $OUT/diag.txt
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
