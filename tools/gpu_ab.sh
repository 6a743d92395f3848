#!/bin/bash
# A/B of two library builds on bench records, alternated twice on one box: the in-tree library (A), then
# KS_LIB_PATH=$1 (B).  $2.. = bench configs (default c2).  Per config and round one line: value, ms/step of A and B.
set -o pipefail
ALT=${1:?usage: tools/gpu_ab.sh ALT_LIB [config ...]}
shift
CFGS=${*:-c2}
OUT=${AB_OUT:-gpurun_out/ab}
mkdir -p $OUT
for r in 1 2; do
  for c in $CFGS; do
    steps=5; [ "$c" = c5 ] && steps=2
    for side in A B; do
      lib=""; [ $side = B ] && lib=$ALT
      KS_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config $c --no-c5 --no-sub --no-cpu-baseline --steps $steps \
        --warmup 1 > $OUT/${c}_${side}_$r.json 2> $OUT/${c}_${side}_$r.err || { tail -5 $OUT/${c}_${side}_$r.err; exit 1; }
    done
    python3 -c "import json;a=json.load(open('$OUT/${c}_A_$r.json'));b=json.load(open('$OUT/${c}_B_$r.json'));print('$c r$r A',a['value'],a['ms_per_step'],'B',b['value'],b['ms_per_step'])"
  done
done
