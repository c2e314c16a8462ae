#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread > gpurun_out/spec_tests.log 2>&1 || { tail -40 gpurun_out/spec_tests.log; exit 1; }
tail -2 gpurun_out/spec_tests.log
timeout -k 10 200 python scripts/exp/spec_skip.py || exit 1
timeout -k 10 200 python scripts/exp/ps_fused.py || exit 1
MODEL=llama400m timeout -k 10 180 python scripts/exp/ab_strategy.py bracket ordered flat || exit 1
