#!/bin/bash
# Round-3: grid encoder with item partials — tests + R18 strategies; Top-K kernel trace at 2048 sampled runs.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py tests/test_gpu_r2.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/r3g_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/exp/r18_strategies.py > gpurun_out/r3g_r18.json 2> gpurun_out/r3g_r18.err || exit 2
rm -rf gpurun_out/r3g_topk_prof
OMF_TOPK_SAMPLE_RUNS=2048 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g_topk_prof -o run -- \
    python3 scripts/exp/tk_runs_sweep.py 2048 > gpurun_out/r3g_topk_prof.log 2>&1 || exit 3
