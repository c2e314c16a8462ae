#!/bin/bash
# Round-3: ResNet-18 kernel trace by launch pattern (which transitions cost an idle gap).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
for pat in edd eed; do
  rm -rf gpurun_out/r3u_$pat
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3u_$pat -o run -- python3 scripts/exp/r18_trace.py - $pat > gpurun_out/r3u_$pat.log 2>&1 || exit 1
  echo "== $pat"; python3 scripts/exp/trace_gaps.py gpurun_out/r3u_$pat 600
done
