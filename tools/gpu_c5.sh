#!/bin/bash
# C5 (1M pods x 100k nodes) bench with CPU baseline, plus rocprofv3 kernel stats of the same command.
set -o pipefail
OUT=gpurun_out/${1:-c5}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --config c5 --steps ${STEPS:-3} --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config c5 --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -30 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
