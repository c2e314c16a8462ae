#!/bin/bash
# Experiment (GPU box): the bucket sort compiled for 6 waves per SIMD (70 VGPRs, 3 workgroups per
# CU) against 8 (64 VGPRs with spills, 4 workgroups per CU): Top-K per-kernel times.
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
d=/tmp/omf_sw8; mkdir -p $d
for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
  timeout -k 10 400 hipcc $F -DOMF_SORT_WAVES=8 -c omnifed_amd/csrc/$s -o $d/$s.o &
done
wait
timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o $d/lib.so $d/*.o || exit 1
run() {
  local o=gpurun_out/tksw_$1; shift; rm -rf $o
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- \
      python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > $o.log 2>&1 || exit 3
}
for rep in 1 2; do
  run w6_$rep OMF_TOPK_SURE=1.5,2
  run w8_$rep OMF_CODEC_LIB_EXPERIMENT=$d/lib.so
done
