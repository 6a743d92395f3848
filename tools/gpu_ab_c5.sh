# A/B of two library builds on the C5 record (1M pods x 100k nodes): default library, then KS_LIB_PATH=$1
set -o pipefail
mkdir -p gpurun_out/ab
ALT=${1:-koordinator_amd/libkoordgpu_prev.so}
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config c5 --no-c5 --no-sub --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/ab/c5base_$r.json 2> gpurun_out/ab/c5base_$r.err || { tail -5 gpurun_out/ab/c5base_$r.err; exit 1; }
  KS_LIB_PATH=$ALT timeout -k 10 300 python -u bench.py --config c5 --no-c5 --no-sub --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/ab/c5alt_$r.json 2> gpurun_out/ab/c5alt_$r.err || { tail -5 gpurun_out/ab/c5alt_$r.err; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/ab/c5base_$r.json'));a=json.load(open('gpurun_out/ab/c5alt_$r.json'));print('c5 base',b['value'],b['ms_per_step'],'alt',a['value'],a['ms_per_step'])"
done
