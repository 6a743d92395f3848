#!/bin/bash
# Parity (shard + basic), commit-phase split for c2/c3/c4, C2 bench and the sweep's PMC traffic.
set -o pipefail
OUT=gpurun_out/${1:-diag}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for C in c2 c3 c4; do
  timeout -k 10 200 python -u tools/diag_commit.py $C > $OUT/diag_$C.txt 2>&1 || { echo "diag $C failed"; tail -20 $OUT/diag_$C.txt; exit 1; }
  cat $OUT/diag_$C.txt
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/pmc_traffic.sh c2 $(basename $OUT)/tr_c2 > /dev/null && python3 -c "import json;t=json.load(open('$OUT/tr_c2/traffic.json'));print({k:v['hbm_bytes_per_launch'] for k,v in t['kernels'].items()})"
