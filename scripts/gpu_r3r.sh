#!/bin/bash
# Round-3: Top-K per-kernel times under two sure-bin margins (rocprofv3 kernel stats).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
for zc in 6,32 1.5,2 1,0; do
  d=gpurun_out/r3r_prof_${zc/,/_}
  rm -rf $d
  OMF_TOPK_SURE=$zc timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > $d.log 2>&1 || exit 3
done
