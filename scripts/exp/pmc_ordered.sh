# PMC traffic (FETCH_SIZE / WRITE_SIZE) of a short bench run, summarised per kernel (helper).
export TMPDIR=/tmp; R=$(pwd); TAG=${1:-pmc}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_$c" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/${TAG}_$c.log; exit 1; }
done
python3 scripts/pmc_traffic.py gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE gpurun_out/${TAG}_traffic.json llama400m 4 && cat gpurun_out/${TAG}_traffic.json
