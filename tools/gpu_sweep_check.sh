#!/bin/bash
# Sweep-kernel change check: parity tests that exercise the Fit + LoadAware sweep, then the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_launch_shape.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); c5=d['c5']
print('C2', d['value'], d['kernel_ms_per_step'], d['roofline']['avg_launch_us']); print('C5', c5['value'], c5['kernel_ms_per_step'], c5['roofline']['avg_launch_us'])"
