#!/bin/bash
# A/B of two source trees on bench records, alternated twice on one box: this tree (A), then the tree at $1 (B: a
# copy of another commit's bench.py, koordinator_amd/ with its built library, and oracle/).  $2.. = bench configs.
set -o pipefail
ALT=${1:?usage: tools/gpu_ab_tree.sh ALT_TREE [config ...]}
shift
CFGS=${*:-c2}
OUT=${AB_OUT:-gpurun_out/abt}
mkdir -p $OUT
for r in 1 2; do
  for c in $CFGS; do
    steps=5; [ "$c" = c5 ] && steps=2
    for side in A B; do
      dir=.; [ $side = B ] && dir=$ALT
      timeout -k 10 300 python -u $dir/bench.py --config $c --no-c5 --no-sub --no-cpu-baseline --steps $steps \
        --warmup 1 > $OUT/${c}_${side}_$r.json 2> $OUT/${c}_${side}_$r.err || { tail -5 $OUT/${c}_${side}_$r.err; exit 1; }
    done
    python3 -c "import json;a=json.load(open('$OUT/${c}_A_$r.json'));b=json.load(open('$OUT/${c}_B_$r.json'));print('$c r$r A',a['value'],a['ms_per_step'],'B',b['value'],b['ms_per_step'])"
  done
done
