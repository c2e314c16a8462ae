#!/bin/bash
# Round-3: grid encoder with Philox words parked in LDS — grid tests, phase costs, R18 strategies.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py -x -q --timeout 200 \
    --timeout-method thread -k "grid or strateg or stream or int8" > gpurun_out/r3j_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/exp/grid_phases.py > gpurun_out/r3j_grid_phases.json 2> gpurun_out/r3j_grid_phases.err || exit 2
timeout -k 10 300 python -u scripts/exp/r18_strategies.py > gpurun_out/r3j_r18.json 2> gpurun_out/r3j_r18.err || exit 3
