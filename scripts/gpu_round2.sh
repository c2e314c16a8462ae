#!/usr/bin/env bash
# Round-2 measurement session (one gpurun call): GPU tests, rocprofv3 kernel stats and PMC
# traffic of a short bench, then the full bench line reading the fresh PMC file.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
T=${TAG:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/${T}_tests.log; exit 1; }
  tail -1 gpurun_out/${T}_tests.log
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/${T}_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${T}_prof.log; exit 1; }
echo "prof ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/${T}_pmc_$c" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${T}_pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/${T}_pmc_$c.log; exit 1; }
done
python3 scripts/pmc_traffic.py gpurun_out/${T}_pmc_FETCH_SIZE gpurun_out/${T}_pmc_WRITE_SIZE gpurun_out/pmc_traffic.json llama400m 4 || exit 1
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 900 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
