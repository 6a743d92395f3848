#!/bin/bash
# rocprofv3 kernel stats for the default bench line (C2), the PMC HBM traffic / VALU-issue passes for C2 and C5
# (C5's sweep measured unpipelined, KS_PIPE=0: the same kernel without the list re-evaluation launches), and last
# the C5 kernel trace (200k pods, patched pipeline) with its overlap summary (tools/trace_overlap.py).  Output
# under gpurun_out/$1, copied into profiles/ by hand.
# A pipelined process under rocprofv3 may segfault at exit after writing its output (the process-lifetime
# CU-masked streams, koordgpu.hip ensure_pipe): the trace step is the last GPU step, and its output is kept only
# when the trace file was written.
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --no-c5 --no-sub --no-cpu-baseline > $OUT/prof_c2.json 2> $OUT/prof_c2.err || { echo "rocprof c2 failed"; tail -30 $OUT/prof_c2.err; exit 1; }
find $OUT/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
echo prof c2 done
BENCH_ARGS="--no-c5 --no-sub" bash tools/pmc_traffic.sh c2 $(basename $OUT)/traffic_c2 || exit 1
BENCH_ARGS="--no-c5 --no-sub" bash tools/pmc_valu.sh c2 $(basename $OUT)/valu_c2 10.8 || exit 1
KS_PIPE=0 BENCH_ARGS="--no-c5 --pods 200000" bash tools/pmc_traffic.sh c5 $(basename $OUT)/traffic_c5 || exit 1
KS_PIPE=0 BENCH_ARGS="--no-c5 --pods 200000" bash tools/pmc_valu.sh c5 $(basename $OUT)/valu_c5 40.3 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config c5 --no-c5 --no-cpu-baseline --pods 200000 --steps 2 --warmup 1 > $OUT/prof_c5.json 2> $OUT/prof_c5.err
rc=$?
TR=$(find $OUT/prof_c5 -name '*kernel_trace.csv' | head -1)
[ -n "$TR" ] && python3 tools/trace_overlap.py $TR > $OUT/c5_overlap.json
find $OUT -type f ! -name '*kernel_stats.csv' ! -name '*.json' ! -name '*.err' -delete
echo "prof c5 trace rc=$rc"
exit 0
