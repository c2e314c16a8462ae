#!/bin/bash
# Round-3: tiled decode A/B (bitmap vs the LDS-cleared tile), interleaved in one process.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/exp/tk_env_ab.py OMF_TOPK_DEC_TILES=lds,bitmap 9 > gpurun_out/r3za_ab.json 2> gpurun_out/r3za_ab.err || { tail -5 gpurun_out/r3za_ab.err; exit 2; }
cat gpurun_out/r3za_ab.json
