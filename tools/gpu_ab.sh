#!/bin/bash
# A/B of the commit-kernel choice for the monotone plugin sets: KS_COMMIT_GENERAL=0 (default: mono kernel without
# ElasticQuota, general kernel with it), =1 (general everywhere), =2 (mono everywhere), after the launch-shape
# parity tests for both choices.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_launch_shape.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/shape.log 2>&1 || { tail -30 gpurun_out/ab/shape.log; exit 1; }
tail -1 gpurun_out/ab/shape.log
for G in ${AB_MODES:-0 2}; do
  KS_COMMIT_GENERAL=$G timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 --c5-pods 200000 > gpurun_out/ab/g$G.json 2> gpurun_out/ab/g$G.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ab/g$G.json')); c5=d['c5']
print('G=$G C2', d['value'], d['kernel_ms_per_step'], 'commit us', d['roofline']['commit']['avg_launch_us'], 'C5', c5['value'], c5['kernel_ms_per_step'])"
done
