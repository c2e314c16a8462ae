#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk_ps.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tk_tests.log 2>&1 || { tail -30 gpurun_out/tk_tests.log; exit 1; }
tail -1 gpurun_out/tk_tests.log
timeout -k 10 200 python scripts/exp/tk_time.py || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d "$(pwd)/gpurun_out/tk_prof" -o run -- python3 "$(pwd)/scripts/exp/tk_time.py" > gpurun_out/tk_prof.log 2>&1 || exit 1
db=$(ls gpurun_out/tk_prof/*/*results.db gpurun_out/tk_prof/*results.db 2>/dev/null | head -1)
python3 scripts/rocpd_stats.py "$db" gpurun_out/tk_stats.csv | grep topk
