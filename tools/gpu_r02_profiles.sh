#!/bin/bash
# Round-2 evidence: the default bench line (C2 + the c5 record + CPU baselines), C3 and C4 lines, and rocprofv3
# kernel stats for C2, C3 and C5 (written under gpurun_out/$1, copied into profiles/ by hand).
set -o pipefail
OUT=gpurun_out/${1:-r02}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail -30 $OUT/bench_c2.err; exit 1; }
echo c2 done
timeout -k 10 400 python -u bench.py --config c3 --no-c5 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -30 $OUT/bench_c3.err; exit 1; }
echo c3 done
timeout -k 10 400 python -u bench.py --config c4 --no-c5 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail -30 $OUT/bench_c4.err; exit 1; }
echo c4 done
for C in c2 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$C -o run -- python3 bench.py --config $C --no-c5 --no-cpu-baseline > $OUT/prof_$C.json 2> $OUT/prof_$C.err || { echo "rocprof $C failed"; tail -30 $OUT/prof_$C.err; exit 1; }
  echo prof $C done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --config c5 --no-c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof_c5.json 2> $OUT/prof_c5.err || { echo "rocprof c5 failed"; tail -30 $OUT/prof_c5.err; exit 1; }
echo prof c5 done
