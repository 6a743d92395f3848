#!/bin/bash
# One library's validation on one MI355X: the -m gpu parity suite, then the c3r / c3rd wall-clock timer
# (tools/c3r_time.py).  Round-end evidence (smoke, bench line, profiles) is tools/gpu_final.sh.
set -o pipefail
O=gpurun_out/${1:-val}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/c3r_time.py 0 0.7 > $O/t.log 2>&1 || { cat $O/t.log; exit 1; }
cat $O/t.log
