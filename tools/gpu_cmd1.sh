# ad-hoc GPU batch of the session
set -o pipefail
mkdir -p gpurun_out/r5f
timeout -k 10 600 python -u -m pytest tests/test_gpu_shipped_profile.py -v -s --timeout 300 --timeout-method thread -k "c3_full" > gpurun_out/r5f/new.log 2>&1
grep -E "PASSED|FAILED|^E .*Error|c3-full:" gpurun_out/r5f/new.log | head -20
timeout -k 10 300 python -u bench.py --config c3f --no-c5 --no-sub --steps 3 --warmup 1 --detail gpurun_out/r5f/c3f_detail.json > gpurun_out/r5f/c3f.json 2> gpurun_out/r5f/c3f.err || { tail -20 gpurun_out/r5f/c3f.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/r5f/c3f.json
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o gpurun_out/r5f/pmc_calib tools/pmc_calib.hip
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r5f/calib/$C -o pmc -- gpurun_out/r5f/pmc_calib > gpurun_out/r5f/calib_$C.log 2>&1 || { tail -5 gpurun_out/r5f/calib_$C.log; exit 1; }
done
python3 tools/pmc_calib.py gpurun_out/r5f/calib > gpurun_out/r5f/pmc_calib.json && cat gpurun_out/r5f/pmc_calib.json
