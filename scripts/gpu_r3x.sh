#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r3x
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r3x -o run -- python3 scripts/exp/tk_step_trace.py > gpurun_out/r3x.log 2>&1 || exit 1
python3 scripts/exp/api_gaps.py gpurun_out/r3x 24
