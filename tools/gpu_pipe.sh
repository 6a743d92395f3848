#!/bin/bash
# Pipelined-pass iteration: the -m gpu parity suite, then C2 + a 200k-pod C5 record with the
# pipeline on and off (A/B).
set -o pipefail
OUT=gpurun_out/${1:-pipe}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for P in 1 0; do
  KS_PIPE=$P timeout -k 10 300 python -u bench.py --no-cpu-baseline --c5-pods ${C5PODS:-200000} ${BENCH_ARGS} > $OUT/bench_p$P.json 2> $OUT/bench_p$P.err || { echo "bench failed"; tail -30 $OUT/bench_p$P.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_p$P.json')); c5=d['c5']
print('PIPE=$P C2', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['passes_per_step'], d['bubble_passes_per_step'])
print('PIPE=$P C5', c5['value'], c5['ms_per_step'], c5['kernel_ms_per_step'], c5['passes_per_step'], c5['bubble_passes_per_step'])"
done
