#!/bin/bash
# bench of one config (arg 2: c2|c3|c4; arg 1: output dir name) with CPU baseline + rocprof kernel stats.
set -o pipefail
CFG=${2:-c4}
OUT=gpurun_out/${1:-$CFG}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config $CFG > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config $CFG --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -30 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
