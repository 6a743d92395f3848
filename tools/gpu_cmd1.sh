# ad-hoc GPU batch of the session: kernel trace of the c2t topology path
set -o pipefail
mkdir -p gpurun_out/r5j
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5j/prof -o c2t -- python3 bench.py --config c2t --no-c5 --no-sub --no-cpu-baseline --no-profile --steps 1 --warmup 0 --pods 2000 > gpurun_out/r5j/bench.json 2> gpurun_out/r5j/bench.err || { tail -20 gpurun_out/r5j/bench.err; exit 1; }
f=$(find gpurun_out/r5j/prof -name "*kernel_stats.csv" | head -1)
head -20 "$f"
