#!/usr/bin/env bash
# Experiment builds of the codec library (never shipped): RNG cost variants.
set -e
cd "$(dirname "$0")/../.."
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
build() {
  local name=$1; shift
  mkdir -p scripts/exp/_build/$name
  for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_topk.hip; do
    hipcc $F "$@" -c omnifed_amd/csrc/$s -o scripts/exp/_build/$name/$s.o &
  done
  wait
  hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/exp/_build/$name/lib.so scripts/exp/_build/$name/*.o
  rm -f scripts/exp/_build/$name/lib.so.*-*
}
build r7 -DOMF_PHILOX_ROUNDS=7
build norng -DOMF_EXP_NORNG
