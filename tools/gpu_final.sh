#!/bin/bash
# Round-end evidence on one MI355X: the -m gpu parity suite, smoke(), the default bench line (C2 + the c5 / c3 / c4
# records with their CPU baselines), then (with PROFILES=1) rocprofv3 kernel stats and PMC traffic / VALU passes
# (tools/gpu_profiles.sh).
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 900 python -u bench.py --detail $OUT/bench_detail.json > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json
if [ "${PROFILES:-0}" = 1 ]; then bash tools/gpu_profiles.sh $(basename $OUT)/prof || exit 1; fi
