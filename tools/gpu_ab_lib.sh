# A/B of two library builds on the C2 bench (the default library, then KS_LIB_PATH=$1), alternated twice
set -o pipefail
mkdir -p gpurun_out/ab
ALT=${1:-koordinator_amd/libkoordgpu_nospec.so}
CFG=${2:-c2}
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config $CFG --no-c5 --no-sub --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab/base_$r.json 2> gpurun_out/ab/base_$r.err || { tail -5 gpurun_out/ab/base_$r.err; exit 1; }
  KS_LIB_PATH=$ALT timeout -k 10 300 python -u bench.py --config $CFG --no-c5 --no-sub --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab/alt_$r.json 2> gpurun_out/ab/alt_$r.err || { tail -5 gpurun_out/ab/alt_$r.err; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/ab/base_$r.json'));a=json.load(open('gpurun_out/ab/alt_$r.json'));print('base',b['value'],b['ms_per_step'],'alt',a['value'],a['ms_per_step'])"
done
