#!/bin/bash
# HBM traffic of the sweep kernel from PMC counters (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE in
# separate passes (TCC slot limits), no tracing domains with --pmc.  arg 1: config (c2|c3|c4|c5|c2d|preempt), arg 2: output dir; BENCH_ARGS: extra bench.py flags (e.g. --pods).
set -o pipefail
CFG=${1:-c2}
OUT=gpurun_out/${2:-traffic_$CFG}
mkdir -p $OUT
export TMPDIR=/tmp
# CFG=preempt: the bench's preempt record alone (bench.py --preempt-only)
if [ "$CFG" = preempt ]; then SEL="--preempt-only"; else SEL="--config $CFG"; fi
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o pmc -- python3 bench.py $SEL --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} > $OUT/$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
python3 tools/traffic.py $OUT $CFG > $OUT/traffic.json && cat $OUT/traffic.json
