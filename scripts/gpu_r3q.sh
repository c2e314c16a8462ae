#!/bin/bash
# Round-3: Top-K sure-bin margin sweep (interleaved A/B; outputs must be identical).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/exp/tk_env_ab.py 'OMF_TOPK_SURE=6:32;1.5:2;6:32;1.5:2' 12 > gpurun_out/r3q_ab.json 2> gpurun_out/r3q_ab.err || { tail -5 gpurun_out/r3q_ab.err; exit 2; }
cat gpurun_out/r3q_ab.json
