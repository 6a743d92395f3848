#!/bin/bash
# the whole -m gpu suite, then the preempt bench record alone
set -o pipefail
OUT=gpurun_out/${1:-tp}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u -c "
import argparse, json, bench
a = argparse.Namespace(preempt_pods=128, cpu_budget_s=10.0)
print(json.dumps(bench.run_preempt(a, 3, 1, True, True)))" > $OUT/preempt.json 2> $OUT/preempt.err || { tail -30 $OUT/preempt.err; exit 1; }
cat $OUT/preempt.json
