#!/usr/bin/env bash
# Spec encoder GPU tests then the strategy timings (experiment; one gpurun call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/spec_tests.log 2>&1 || { tail -40 gpurun_out/spec_tests.log; exit 1; }
tail -2 gpurun_out/spec_tests.log
bash scripts/exp/spec_perf.sh
