#!/bin/bash
# Round-3 final: the whole GPU suite and smoke() on the committed sources.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_tests.log 2>&1 || { tail -30 gpurun_out/r03_tests.log; exit 1; }
tail -1 gpurun_out/r03_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1 || { tail -5 gpurun_out/r03_smoke.log; exit 2; }
tail -1 gpurun_out/r03_smoke.log
