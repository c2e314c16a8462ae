#!/bin/bash
# Round-3: grid encoder phase costs (ResNet-18 s = 3).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/exp/grid_phases.py > gpurun_out/r3h_grid_phases.json 2> gpurun_out/r3h_grid_phases.err || exit 1
