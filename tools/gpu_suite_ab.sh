#!/bin/bash
# The whole -m gpu suite, then an A/B of bench settings (tools/gpu_ab_envs.sh arguments after the output dir).
set -o pipefail
OUT=gpurun_out/${1:-suite}
shift 1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -v "^  File\|^    " $OUT/pytest_gpu.log | tail -40; exit 1; }
tail -1 $OUT/pytest_gpu.log
[ $# -gt 0 ] && bash tools/gpu_ab_envs.sh $(basename $OUT)/ab "$@"
exit 0
