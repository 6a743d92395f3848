#!/bin/bash
# preemption GPU parity tests, then the bench's preempt record alone (bench.py --preempt-only)
set -o pipefail
OUT=gpurun_out/${1:-pq}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_preempt.py tests/test_gpu_refusals.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u bench.py --preempt-only --steps 3 --warmup 1 --no-cpu-baseline > $OUT/preempt.json 2> $OUT/preempt.err || { tail -20 $OUT/preempt.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/preempt.json'))['preempt']; print(d['value'], d['us_per_preemption'], d['roofline'])"
