set -o pipefail
O=gpurun_out/${1:-r06h}; mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 1000 python -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python3 tools/bench_summary.py $O/bench.json
