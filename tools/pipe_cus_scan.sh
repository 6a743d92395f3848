#!/bin/bash
# C5 (200k-pod queue) under several commit-stream CU counts (KS_PIPE_COMMIT_CUS; the sweep stream gets the rest)
set -o pipefail
OUT=gpurun_out/pipe_cus
mkdir -p $OUT
for c in ${CUS:-16 32 48 64}; do
  KS_PIPE_COMMIT_CUS=$c timeout -k 10 240 python -u bench.py --config c5 --pods 200000 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-sub --no-c5 > $OUT/c$c.json 2> $OUT/c$c.err || { tail -20 $OUT/c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernel_ms_per_step'])" $OUT/c$c.json $c
done
