#!/bin/bash
# rocprofv3 kernel stats for the default bench line (C2) and C5, and the PMC HBM
# traffic / VALU-issue passes for C2 and C5 (written under gpurun_out/$1, copied into profiles/ by hand).
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --no-c5 --no-sub --no-cpu-baseline > $OUT/prof_c2.json 2> $OUT/prof_c2.err || { echo "rocprof c2 failed"; tail -30 $OUT/prof_c2.err; exit 1; }
find $OUT/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
echo prof c2 done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config c5 --no-c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof_c5.json 2> $OUT/prof_c5.err || { echo "rocprof c5 failed"; tail -30 $OUT/prof_c5.err; exit 1; }
find $OUT/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
echo prof c5 done
BENCH_ARGS="--no-c5 --no-sub" bash tools/pmc_traffic.sh c2 $(basename $OUT)/traffic_c2 || exit 1
BENCH_ARGS="--no-c5 --pods 200000" bash tools/pmc_traffic.sh c5 $(basename $OUT)/traffic_c5 || exit 1
BENCH_ARGS="--no-c5 --pods 200000" bash tools/pmc_valu.sh c5 $(basename $OUT)/valu_c5 40.3 || exit 1
BENCH_ARGS="--no-c5 --no-sub" bash tools/pmc_valu.sh c2 $(basename $OUT)/valu_c2 10.8 || exit 1
# keep the summaries only (gpurun copies back at most 64 MiB)
find $OUT -type f ! -name '*kernel_stats.csv' ! -name '*.json' ! -name '*.err' -delete
