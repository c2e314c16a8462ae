#!/bin/bash
# Round-3 measurements on the committed sources: rocprofv3 kernel stats of the bench (QSGD line and
# the Top-K line), the two PMC passes (FETCH_SIZE, WRITE_SIZE; QSGD and Top-K launches of the same
# bench), the full bench line (reads the fresh PMC file), and the host-inclusive wire path.
# OMF_COMMIT names the commit (the box's copy has no .git).  Results are copied into profiles/.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
R=$(pwd)
T=${OMF_TAG:-r03}
mkdir -p gpurun_out
rm -rf gpurun_out/${T}_prof gpurun_out/${T}_topk_prof gpurun_out/${T}_pmc_FETCH_SIZE gpurun_out/${T}_pmc_WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_prof" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/${T}_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${T}_prof.log; exit 1; }
echo "prof ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_topk_prof" -o run -- python3 "$R/bench.py" --codec topk --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/${T}_topk_prof.log 2>&1 || { echo "topk prof failed"; tail -5 gpurun_out/${T}_topk_prof.log; exit 1; }
echo "topk prof ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/${T}_pmc_$c" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${T}_pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/${T}_pmc_$c.log; exit 2; }
done
python3 scripts/pmc_traffic.py gpurun_out/${T}_pmc_FETCH_SIZE gpurun_out/${T}_pmc_WRITE_SIZE gpurun_out/pmc_traffic.json llama400m 4 || exit 3
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 600 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.err; exit 4; }
cat gpurun_out/${T}_bench.json
timeout -k 10 300 python3 -u scripts/wire_bench.py > gpurun_out/${T}_wire.json 2> gpurun_out/${T}_wire.err || { echo "wire failed"; exit 5; }
timeout -k 10 300 python3 -u scripts/wire_breakdown.py > gpurun_out/${T}_wire_breakdown.json 2> gpurun_out/${T}_wire_breakdown.err || { echo "breakdown failed"; exit 6; }
for f in ${T}_prof ${T}_topk_prof; do
  s=$(find gpurun_out/$f -name '*kernel_stats.csv' | head -n 1)
  [ -n "$s" ] && cp "$s" profiles/${f/_prof/}_kernel_stats.csv
done
cp gpurun_out/${T}_bench.json profiles/${T}_bench.json
cp gpurun_out/${T}_wire.json profiles/${T}_wire.json
cp gpurun_out/${T}_wire_breakdown.json profiles/${T}_wire_breakdown.json
mkdir -p gpurun_out/profiles_copy && cp profiles/pmc_traffic.json profiles/${T}_* gpurun_out/profiles_copy/
echo "measure ok"
