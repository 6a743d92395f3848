#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/kvar
for K in 8 16 24 32 48; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --candidates $K > gpurun_out/kvar/c2_k$K.json 2> gpurun_out/kvar/err_$K.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/kvar/c2_k$K.json'));print('c2 K=$K', d['value'], d['kernel_ms_per_step'], d['passes_per_step'], d['cut_passes_per_step'], d['rescans_per_step'])"
done
for K in 16 32; do
  timeout -k 10 120 python -u bench.py --config c3 --no-cpu-baseline --candidates $K > gpurun_out/kvar/c3_k$K.json 2> gpurun_out/kvar/err3_$K.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/kvar/c3_k$K.json'));print('c3 K=$K', d['value'], d['kernel_ms_per_step'], d['passes_per_step'], d['cut_passes_per_step'], d['rescans_per_step'])"
done
