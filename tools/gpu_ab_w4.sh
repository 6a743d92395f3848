#!/bin/bash
# A/B of library builds (KS_LIB_PATH) on C2 + a 200k-pod C5 step: value, kernel split and sweep launch time.
set -o pipefail
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
shift
for lib in "$@"; do
  KS_LIB_PATH=$PWD/koordinator_amd/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-sub --c5-pods 200000 --steps 5 --warmup 2 > $OUT/$lib.json 2>$OUT/$lib.err || { echo "$lib failed"; tail -5 $OUT/$lib.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$lib.json')); c=d['c5']
print('$lib', 'C2', d['value'], d['kernel_ms_per_step'], d['roofline']['avg_launch_us'], '| C5', c['value'], c['ms_per_step'], c['kernel_ms_per_step'], c['roofline']['avg_launch_us'])"
done
