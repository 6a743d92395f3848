#!/bin/bash
# A/B of environment settings on the default bench line (C2 + the c5 record, no c3 / c4, no CPU baseline):
# arg 1 output dir, arg 2.. settings, each "VAR=value[:VAR=value...]"; PYTEST_K: run these -m gpu tests first.
set -o pipefail
OUT=gpurun_out/${1:-ab}
shift 1
mkdir -p $OUT
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
i=0
for V in "$@"; do
  i=$((i+1))
  env $(echo $V | tr ':' ' ') timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-sub --c5-pods ${C5PODS:-200000} ${BENCH_ARGS} > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench failed"; tail -30 $OUT/bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$i.json')); c5=d['c5']
print('$V C2', d['value'], d['ms_per_step'])
print('$V C5', c5['value'], c5['ms_per_step'], c5['kernel_ms_per_step'], c5['passes_per_step'], c5['pipelined'])"
done
