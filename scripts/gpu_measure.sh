#!/usr/bin/env bash
# One measurement session on the GPU box: bench line, rocprofv3 kernel stats, and the two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for per-launch HBM traffic.  Every GPU step
# is time-bounded and the steps are chained: a failure ends the session.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/prof.log 2>&1
echo "stats ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$c" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/pmc_$c.log 2>&1
done
python3 scripts/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_traffic.json
