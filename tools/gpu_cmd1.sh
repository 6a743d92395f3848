# ad-hoc GPU batch of the session
set -o pipefail
mkdir -p gpurun_out/r5h
timeout -k 10 900 python -u -m pytest tests/test_gpu_topology.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5h/topo.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E .*Error|^E  " gpurun_out/r5h/topo.log | head -60
exit $rc
