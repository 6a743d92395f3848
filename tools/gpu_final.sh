#!/bin/bash
# Round-end evidence on one MI355X: the -m gpu parity suite, smoke(), the default bench line (C2 + c5 record + CPU
# baselines), C3 / C4 lines, then rocprofv3 kernel stats and PMC traffic / VALU passes (tools/gpu_r02b_profiles.sh).
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); c5=d['c5']
print('C2', d['value'], d['parity'], d['kernel_ms_per_step'], 'cpu', d['cpu_baseline']['value'])
print('C5', c5['value'], c5['parity'], c5['kernel_ms_per_step'], 'cpu', c5['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --config c3 --no-c5 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -30 $OUT/bench_c3.err; exit 1; }
timeout -k 10 400 python -u bench.py --config c4 --no-c5 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail -30 $OUT/bench_c4.err; exit 1; }
python3 -c "
import json
for c in ('c3', 'c4'):
    d=json.load(open('$OUT/bench_'+c+'.json')); print(c, d['value'], d['parity'], d['kernel_ms_per_step'], 'cpu', d['cpu_baseline']['value'])"
