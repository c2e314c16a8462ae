#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -40 gpurun_out/dec_tests.log; exit 1; }
tail -2 gpurun_out/dec_tests.log
timeout -k 10 200 python scripts/exp/dec_vs_probe.py || exit 1
