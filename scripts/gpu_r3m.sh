#!/bin/bash
# Round-3: fine-bin histogram counted in the fused pass — Top-K tests and the interleaved A/B.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk_ps.py tests/test_gpu_r3.py tests/test_gpu_r2.py -x -q --timeout 200 \
    --timeout-method thread -k "topk or Topk or TopK" > gpurun_out/r3m_tests.log 2>&1 || { tail -20 gpurun_out/r3m_tests.log; exit 1; }
tail -1 gpurun_out/r3m_tests.log
timeout -k 10 300 python -u scripts/exp/tk_env_ab.py OMF_TOPK_FUSED_HIST=0,1 7 > gpurun_out/r3m_ab.json 2> gpurun_out/r3m_ab.err || { tail -5 gpurun_out/r3m_ab.err; exit 2; }
cat gpurun_out/r3m_ab.json
