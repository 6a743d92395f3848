#!/bin/bash
# Profile evidence of the bench line's records, all from the library in this tree (each summary is stamped with its
# sha256, which bench.py checks): per config (c2, c3, c4, c2d, c2s, c3r, c3rd) the rocprofv3 kernel statistics of the bench command and
# the PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and VALU-issue summaries; for c5 the PMC passes on a 200k-pod
# queue (sweep measured unpipelined, KS_PIPE=0: the same kernel without the list re-evaluation launches) and last the
# pipelined kernel trace with its overlap summary (tools/trace_overlap.py).
# Output: gpurun_out/$1/<cfg>_{kernel_stats.csv,traffic.json,valu.json}, preempt_{kernel_stats.csv,traffic.json},
# c5_overlap.json; tools/keep_profiles.sh copies
# them into profiles/ under a round tag.
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
for CFG in ${CONFIGS:-c2 c3 c4 c2d c2s c3r c3rd}; do
  # (c2d: the topology loop without its HIP graph -- rocprofv3's CSV kernel trace of the captured loop died in the
  # HIP runtime in round 5)
  G=1; [ "$CFG" = c2d ] && G=0
  KS_TOPO_GRAPH=$G timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$CFG -o run -- python3 bench.py --config $CFG --no-c5 --no-sub --no-cpu-baseline > $OUT/prof_$CFG.json 2> $OUT/prof_$CFG.err || { echo "rocprof $CFG failed"; tail -30 $OUT/prof_$CFG.err; exit 1; }
  S=$(find $OUT/prof_$CFG -name '*kernel_stats.csv' | head -1)
  [ -n "$S" ] && cp $S $OUT/${CFG}_kernel_stats.csv
  rm -rf $OUT/prof_$CFG
  # (c2d's PMC passes on 1,000 pods: --pmc serializes each of the ~4 dispatches per topology pod)
  PARGS="--no-c5 --no-sub"; [ "$CFG" = c2d ] && PARGS="$PARGS --pods 1000"
  BENCH_ARGS="$PARGS" bash tools/pmc_traffic.sh $CFG ${OUT#gpurun_out/}/traffic_$CFG > /dev/null || exit 1
  cp $OUT/traffic_$CFG/traffic.json $OUT/${CFG}_traffic.json
  BENCH_ARGS="$PARGS" bash tools/pmc_valu.sh $CFG ${OUT#gpurun_out/}/valu_$CFG > /dev/null || exit 1
  cp $OUT/valu_$CFG/valu.json $OUT/${CFG}_valu.json
  rm -rf $OUT/traffic_$CFG $OUT/valu_$CFG
  echo "profiles $CFG done"
done
if [ "${PREEMPT:-1}" = 1 ]; then
  # the PostFilter kernels (bench.py --preempt-only): kernel statistics and PMC HBM traffic
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_preempt -o run -- python3 bench.py --preempt-only --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_preempt.json 2> $OUT/prof_preempt.err || { echo "rocprof preempt failed"; tail -30 $OUT/prof_preempt.err; exit 1; }
  S=$(find $OUT/prof_preempt -name '*kernel_stats.csv' | head -1)
  [ -n "$S" ] && cp $S $OUT/preempt_kernel_stats.csv
  rm -rf $OUT/prof_preempt
  bash tools/pmc_traffic.sh preempt ${OUT#gpurun_out/}/traffic_preempt > /dev/null || exit 1
  cp $OUT/traffic_preempt/traffic.json $OUT/preempt_traffic.json
  rm -rf $OUT/traffic_preempt
  echo "profiles preempt done"
fi
if [ "${C5:-1}" = 1 ]; then
  KS_PIPE=0 BENCH_ARGS="--no-c5 --pods 200000" bash tools/pmc_traffic.sh c5 ${OUT#gpurun_out/}/traffic_c5 > /dev/null || exit 1
  cp $OUT/traffic_c5/traffic.json $OUT/c5_traffic.json
  KS_PIPE=0 BENCH_ARGS="--no-c5 --pods 200000" bash tools/pmc_valu.sh c5 ${OUT#gpurun_out/}/valu_c5 > /dev/null || exit 1
  cp $OUT/valu_c5/valu.json $OUT/c5_valu.json
  rm -rf $OUT/traffic_c5 $OUT/valu_c5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config c5 --no-c5 --no-cpu-baseline --pods 200000 --steps 2 --warmup 1 > $OUT/prof_c5.json 2> $OUT/prof_c5.err
  rc=$?
  S=$(find $OUT/prof_c5 -name '*kernel_stats.csv' | head -1)
  [ -n "$S" ] && cp $S $OUT/c5_kernel_stats.csv
  TR=$(find $OUT/prof_c5 -name '*kernel_trace.csv' | head -1)
  [ -n "$TR" ] && python3 tools/trace_overlap.py $TR > $OUT/c5_overlap.json
  rm -rf $OUT/prof_c5
  echo "profiles c5 done (trace rc=$rc)"
fi
exit 0
