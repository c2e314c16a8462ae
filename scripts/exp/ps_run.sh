#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_spec.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ps_tests.log 2>&1 || { tail -30 gpurun_out/ps_tests.log; exit 1; }
tail -1 gpurun_out/ps_tests.log
timeout -k 10 200 python scripts/exp/ps_fused.py || exit 1
