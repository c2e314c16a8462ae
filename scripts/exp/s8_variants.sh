#!/usr/bin/env bash
# Wide-level (s = 8) bracketed encoder variants, Llama-400M: experiment builds of the library
# (never shipped) differing in the bracket's workgroups per tensor (OMF_BR_PARTS) and the fix
# threads per wave slot (OMF_FIX_FT), plus the bracket width in sigmas (OMF_SPEC_ZSIG, runtime);
# each timed by scripts/exp/enc_time.py (HIP events, median of rounds), two interleaved passes.
# Build here:  bash scripts/exp/s8_variants.sh build    Run on the GPU box:  bash scripts/exp/s8_variants.sh run
set -e
cd "$(dirname "$0")/../.."
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
V="base:-DOMF_BR_PARTS=2 p4:-DOMF_BR_PARTS=4 p1:-DOMF_BR_PARTS=1 ft2:-DOMF_FIX_FT=2 ft8:-DOMF_FIX_FT=8"
if [ "$1" = build ]; then
  for v in $V; do
    name=${v%%:*}; flags=${v#*:}
    mkdir -p exp_libs/$name
    for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
      hipcc $F $flags -c omnifed_amd/csrc/$s -o exp_libs/$name/$s.o &
    done
    wait
    hipcc --offload-arch=gfx950 -shared -fPIC -o exp_libs/$name/lib.so exp_libs/$name/*.o
    rm -f exp_libs/$name/*.o exp_libs/$name/lib.so.*-*
  done
  exit 0
fi
for pass in 1 2; do
  for v in $V; do
    name=${v%%:*}
    OMF_CODEC_LIB_EXPERIMENT=exp_libs/$name/lib.so timeout -k 10 120 python3 scripts/exp/enc_time.py llama400m 8 \
      | sed "s/^/{\"variant\": \"$name\", \"pass\": $pass, \"r\": /; s/$/}/"
  done
  for z in 5 4; do
    OMF_SPEC_ZSIG=$z OMF_CODEC_LIB_EXPERIMENT=exp_libs/base/lib.so timeout -k 10 120 python3 scripts/exp/enc_time.py llama400m 8 \
      | sed "s/^/{\"variant\": \"zsig$z\", \"pass\": $pass, \"r\": /; s/$/}/"
  done
done
