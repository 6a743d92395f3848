#!/bin/bash
# VALU issue of the sweep from one PMC pass (8 SQ counters + 1 GRBM, within gfx950's per-pass slots;
# no tracing domains with --pmc).  arg 1: config, arg 2: output dir, arg 3: un-instrumented sweep
# launch time in us (for the fraction); BENCH_ARGS: extra bench.py flags (e.g. --pods).
set -o pipefail
CFG=${1:-c5}
OUT=gpurun_out/${2:-valu_$CFG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/pmc -o pmc -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 tools/valu.py $OUT/pmc $CFG $3 > $OUT/valu.json && cat $OUT/valu.json
