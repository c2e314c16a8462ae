#!/bin/bash
# Round-3: grid encoder tests + strategy timings, wire breakdown, Top-K bench + kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/r3d_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/exp/r18_strategies.py > gpurun_out/r3d_r18.json 2> gpurun_out/r3d_r18.err || exit 2
timeout -k 10 200 python -u scripts/wire_breakdown.py > gpurun_out/r3d_wire_breakdown.json 2>&1 || exit 3
OMF_TOPK_DBG=4 timeout -k 10 300 python -u bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 \
    > gpurun_out/r3d_topk_bench.json 2> gpurun_out/r3d_topk_bench.err || exit 4
rm -rf gpurun_out/r3d_topk_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3d_topk_prof -o run -- \
    python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 10 > gpurun_out/r3d_topk_prof.log 2>&1 || exit 5
