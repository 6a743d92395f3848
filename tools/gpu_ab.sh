set -o pipefail
mkdir -p gpurun_out/ab
for G in 0 1; do
  KS_COMMIT_GENERAL=$G timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 --c5-pods 200000 > gpurun_out/ab/g$G.json 2> gpurun_out/ab/g$G.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab/g$G.json')); c5=d['c5']
print('G=$G C2', d['value'], d['kernel_ms_per_step'], 'commit us', d['roofline']['commit']['avg_launch_us'], 'C5', c5['value'], c5['kernel_ms_per_step'])"
done
