#!/bin/bash
# Round-3: group pipeline with the streaming passes chained across the two streams — tests, A/B.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_r3.py -x -q --timeout 200 --timeout-method thread \
    -k "group_pipeline" > gpurun_out/r3o_tests.log 2>&1 || { tail -20 gpurun_out/r3o_tests.log; exit 1; }
tail -1 gpurun_out/r3o_tests.log
timeout -k 10 400 python -u scripts/exp/tk_env_ab.py OMF_TOPK_GROUPS=1,2,3,4,6,8 7 > gpurun_out/r3o_ab.json 2> gpurun_out/r3o_ab.err || { tail -5 gpurun_out/r3o_ab.err; exit 2; }
cat gpurun_out/r3o_ab.json
