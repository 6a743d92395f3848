#!/bin/bash
# Time C2 with several builds of libkoordgpu (KS_LIB_PATH), commit-kernel A/B.
set -o pipefail
OUT=gpurun_out/${1:-v}
mkdir -p $OUT
shift
for lib in "$@"; do
  KS_LIB_PATH=$PWD/koordinator_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-c5 --steps 3 --warmup 1 > $OUT/$lib.json 2>$OUT/$lib.err || { echo "$lib failed"; tail -5 $OUT/$lib.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$lib.json')); print('$lib', d['value'], d['kernel_ms_per_step'], d['roofline']['commit']['cycles_per_pod'])"
done
