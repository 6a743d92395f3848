# ad-hoc GPU batch of the session
set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 600 python -u -m pytest tests/test_gpu_shipped_profile.py tests/test_gpu_reservation.py tests/test_gpu_deviceshare.py -v --timeout 300 --timeout-method thread > gpurun_out/r5d/new.log 2>&1
grep -E "PASSED|FAILED|^E .*Error" gpurun_out/r5d/new.log | head -60
