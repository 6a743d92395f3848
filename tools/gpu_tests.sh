#!/bin/bash
# GPU parity tests (optionally a subset: $2 = pytest -k expression), then smoke().
set -o pipefail
OUT=gpurun_out/${1:-t}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${2:+-k} ${2:+"$2"} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
