#!/bin/bash
# PMC counters for the C2 kernels (one pass per counter group; no tracing domains combined with --pmc), averaged
# per dispatch of each kernel (tools/pmc_summary.py).
set -o pipefail
OUT=gpurun_out/${1:-pmc}
CFG=${2:-c2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv -d $OUT/p1 -o p1 -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-c5 --no-cpu-baseline > $OUT/p1.log 2>&1 || { echo "pmc1 failed"; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $OUT/p2 -o p2 -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-c5 --no-cpu-baseline > $OUT/p2.log 2>&1 || { echo "pmc2 failed"; tail -5 $OUT/p2.log; exit 1; }
python3 tools/pmc_summary.py $OUT commit
