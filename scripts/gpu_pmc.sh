#!/usr/bin/env bash
# Two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench, kernel-trace only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$c" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_$c.log; exit 1; }
done
python3 scripts/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_traffic.json
