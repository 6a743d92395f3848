#!/bin/bash
# One iteration on the GPU box: the -m gpu parity suite, smoke(), the default bench line (C2 + the c5 record),
# and the commit kernel's per-category cycles (libkoordgpu_cat.so, tools/build_diag.sh) for C2 and C5.
set -o pipefail
OUT=gpurun_out/${1:-it}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
c5=d.get('c5') or {}
print('C2', d['value'], d['kernel_ms_per_step'], 'sweep us', d['roofline']['avg_launch_us'], 'commit us', d['roofline']['commit']['avg_launch_us'], 'cyc/pod', d['roofline']['commit']['cycles_per_pod'])
print('C5', c5.get('value'), c5.get('kernel_ms_per_step'), (c5.get('roofline') or {}).get('avg_launch_us'))
"
if [ -f koordinator_amd/libkoordgpu_seg.so ]; then
  for C in c2 c5; do
    timeout -k 10 200 python -u tools/diag_commit.py $C --seg > $OUT/seg_$C.txt 2>&1 || { echo "seg $C failed"; tail -20 $OUT/seg_$C.txt; exit 1; }
    cat $OUT/seg_$C.txt
  done
fi
if [ -f koordinator_amd/libkoordgpu_cat.so ]; then
  for C in c2 c5; do
    timeout -k 10 200 python -u tools/diag_commit.py $C --cat > $OUT/cat_$C.txt 2>&1 || { echo "cat $C failed"; tail -20 $OUT/cat_$C.txt; exit 1; }
    cat $OUT/cat_$C.txt
  done
fi
if [ -f koordinator_amd/libkoordgpu_cat.so ] && [ -n "$ITER_C3" ]; then
  timeout -k 10 200 python -u tools/diag_commit.py c3 --cat > $OUT/cat_c3.txt 2>&1 || { echo "cat c3 failed"; tail -20 $OUT/cat_c3.txt; exit 1; }
  cat $OUT/cat_c3.txt
fi
