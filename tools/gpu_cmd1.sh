# ad-hoc GPU batch of the session
set -o pipefail
mkdir -p gpurun_out/r5g
timeout -k 10 900 python -u -m pytest tests/test_gpu_numa_bind.py tests/test_gpu_cpu_bind.py tests/test_gpu_c3_policy.py tests/test_gpu_shipped_profile.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r5g/new.log 2>&1
grep -E "PASSED|FAILED|^E .*Error|c3-full:" gpurun_out/r5g/new.log | head -60
timeout -k 10 300 python -u bench.py --config c3f --no-c5 --no-sub --steps 3 --warmup 1 --detail gpurun_out/r5g/c3f_detail.json > gpurun_out/r5g/c3f.json 2> gpurun_out/r5g/c3f.err || { tail -20 gpurun_out/r5g/c3f.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/r5g/c3f.json
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o gpurun_out/r5g/pmc_calib tools/pmc_calib.hip
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r5g/calib/$C -o pmc -- gpurun_out/r5g/pmc_calib > gpurun_out/r5g/calib_$C.log 2>&1 || { tail -5 gpurun_out/r5g/calib_$C.log; exit 1; }
done
python3 tools/pmc_calib.py gpurun_out/r5g/calib > gpurun_out/r5g/pmc_calib.json && cat gpurun_out/r5g/pmc_calib.json
