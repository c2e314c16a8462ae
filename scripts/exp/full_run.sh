#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -40 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 200 python scripts/exp/spec_skip.py || exit 1
MODEL=llama400m timeout -k 10 180 python scripts/exp/ab_strategy.py bracket ordered flat || exit 1
timeout -k 10 200 python scripts/exp/ps_fused.py || exit 1
