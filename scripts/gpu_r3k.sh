#!/bin/bash
# Round-3: Top-K super-item table + staged fine-bin map — Top-K tests, timing, kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk_ps.py tests/test_gpu_r3.py tests/test_gpu_r2.py -x -q --timeout 200 \
    --timeout-method thread -k "topk or Topk or TopK" > gpurun_out/r3k_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/exp/tk_runs_sweep.py 2048 4096 > gpurun_out/r3k_sweep.json 2> gpurun_out/r3k_sweep.err || exit 2
rm -rf gpurun_out/r3k_topk_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k_topk_prof -o run -- \
    python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 10 > gpurun_out/r3k_topk_prof.log 2>&1 || exit 3
