set -o pipefail
bash tools/gpu_quick.sh q3 &&
timeout -k 10 200 python tools/diag_commit.py c2 > gpurun_out/q3/diag.log 2>&1 &&
timeout -k 10 200 python tools/diag_commit.py c4 >> gpurun_out/q3/diag.log 2>&1
