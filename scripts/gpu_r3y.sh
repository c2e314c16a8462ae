#!/bin/bash
# Round-3: Top-K per-kernel times against the sample size (runs per tensor at most).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
for runs in 2048 1024 512; do
  d=gpurun_out/r3y_prof_$runs
  rm -rf $d
  OMF_TOPK_SAMPLE_RUNS=$runs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > $d.log 2>&1 || exit 3
done
