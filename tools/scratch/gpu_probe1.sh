#!/bin/bash
set -o pipefail
OUT=gpurun_out/probe1; mkdir -p $OUT
timeout -k 10 90 python -u tools/scratch/cumask_probe.py 300 > $OUT/probe.log 2>&1; echo "probe rc=$?"; tail -3 $OUT/probe.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1; echo "parity rc=$?"; grep -E "PASS|FAIL|Timeout" $OUT/parity.log | tail -30
