#!/bin/bash
# Llama-400M bf16 / fp16 encodes: the bracketed encoder (the plan's default) against the two-pass.
set -o pipefail
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
for f in 1 2; do
  for st in bracket ordered; do
    timeout -k 10 200 python3 scripts/exp/enc_time.py llama400m 4 $st $f 0 >> gpurun_out/half_enc.txt 2>> gpurun_out/half_enc.err || exit 2
  done
done
cat gpurun_out/half_enc.txt
