#!/bin/bash
# Sweep launch-shape scan: bench.py for one config under several (pods per wave, block cap) settings
# (KS_SWEEP_PPW / KS_SWEEP_BLOCK_CAP, read by ks_schedule); prints pods/s and the sweep's ms per step.
# usage: tools/sweep_shape.sh <config> "<ppw>:<cap> ..."   (ppw 0 = the built-in heuristic)
set -o pipefail
CFG=${1:-c5}
SHAPES=${2:-"0:2048 0:1024 8:1024 8:2048 4:2048 32:2048"}
OUT=gpurun_out/shape_$CFG
mkdir -p $OUT
for s in $SHAPES; do
  ppw=${s%%:*}; cap=${s##*:}
  KS_SWEEP_PPW=$ppw KS_SWEEP_BLOCK_CAP=$cap timeout -k 10 240 python -u bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 \
    --no-cpu-baseline > $OUT/b_${ppw}_${cap}.json 2> $OUT/b_${ppw}_${cap}.err || { echo "bench $s failed"; tail -20 $OUT/b_${ppw}_${cap}.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['kernel_ms_per_step'], d['roofline']['avg_launch_us'], d.get('parity'))" \
    $OUT/b_${ppw}_${cap}.json "$s"
done
