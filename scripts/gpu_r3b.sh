#!/bin/bash
# Round-3 check: wire breakdown, Top-K bench with rotating gradients (+ fallback census), wire tests.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_packed_wire.py tests/test_gpu_integration.py \
    tests/test_gpu_r3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/wire_breakdown.py > gpurun_out/r3b_wire_breakdown.json 2> gpurun_out/r3b_wire_breakdown.err || exit 2
OMF_TOPK_DBG=4 timeout -k 10 300 python -u bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 \
    > gpurun_out/r3b_topk_bench.json 2> gpurun_out/r3b_topk_bench.err || exit 3
timeout -k 10 300 python -u scripts/wire_bench.py > gpurun_out/r3b_wire.json 2> gpurun_out/r3b_wire.err || exit 4
