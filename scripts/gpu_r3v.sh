#!/bin/bash
# Round-3: idle gap after the finish launch with and without its polling fix phase.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
for sp in 24 0; do
  rm -rf gpurun_out/r3v_$sp
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3v_$sp -o run -- python3 scripts/exp/gap_probe.py $sp > gpurun_out/r3v_$sp.log 2>&1 || exit 1
  echo "== spec $sp"; python3 scripts/exp/trace_gaps.py gpurun_out/r3v_$sp 120
done
