#!/bin/bash
# preemption (ks_preempt) GPU parity tests, then the bench's preempt record alone (with its CPU baseline)
set -o pipefail
OUT=gpurun_out/${1:-pre}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_preempt.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u -c "
import argparse, json, bench
a = argparse.Namespace(preempt_pods=128, cpu_budget_s=10.0)
print(json.dumps(bench.run_preempt(a, 3, 1, True, True)))" > $OUT/preempt.json 2> $OUT/preempt.err || { tail -30 $OUT/preempt.err; exit 1; }
cat $OUT/preempt.json
