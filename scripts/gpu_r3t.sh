#!/bin/bash
# Round-3: ResNet-18 step kernel trace (ring and grid encoders): durations and idle gaps.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
for st in ring grid; do
  rm -rf gpurun_out/r3t_$st
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3t_$st -o run -- python3 scripts/exp/r18_trace.py $st > gpurun_out/r3t_$st.log 2>&1 || exit 1
  echo "== $st"; python3 scripts/exp/trace_gaps.py gpurun_out/r3t_$st 400
done
