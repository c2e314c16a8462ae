# GPU tests (all), then a short bench and its rocprof kernel stats (experiment helper).
export TMPDIR=/tmp; R=$(pwd); TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1; tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
python3 scripts/rocpd_stats.py $(find gpurun_out/${TAG}_prof -name "*.db" | head -1) gpurun_out/${TAG}_stats.csv
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
