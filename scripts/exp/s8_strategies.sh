#!/bin/bash
# Llama-400M encoders for what the bracketed encoder does not serve (s > 4, bf16 / fp16 values,
# caller uniforms): the two-pass encoder ("ordered") against the single-read ring, interleaved.
set -o pipefail
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
for args in "8 X 0 0" "4 X 1 0" "4 X 0 1" "8 X 0 0"; do
  for st in ordered ring; do
    set -- $args
    timeout -k 10 200 python3 scripts/exp/enc_time.py llama400m $1 $st $3 $4 >> gpurun_out/s8_ab.txt 2>> gpurun_out/s8_ab.err || exit 2
  done
done
cat gpurun_out/s8_ab.txt
