#!/bin/bash
# C4 (20k nodes, 50k reservations) bench with CPU baseline + rocprof kernel stats.
set -o pipefail
OUT=gpurun_out/${1:-c4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config c4 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config c4 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -30 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
