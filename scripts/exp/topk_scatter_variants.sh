#!/usr/bin/env bash
# Top-K fine-histogram / bucket-scatter variants, Llama-400M k = 1 %: experiment builds of the
# library (never shipped) differing in the keys per thread kept in registers between the scatter's
# count and place phases (OMF_SCATTER_CACHE x 4) and the fine histogram's key loads in flight per
# thread (OMF_FHIST_U) and the bucket sort's sub-bins (OMF_SORT_LOCAL: an LDS histogram of the
# bucket's keys, or the fine bins) and waves per SIMD (OMF_SORT_WAVES), and the fine bins' expected
# fill (OMF_FINE_MARGIN: a fine bin expects <= 2048 / margin candidates); each profiled by rocprofv3 --kernel-trace --stats over
# the bench's Top-K line (per-kernel averages -> gpurun_out/tks_<variant>_kernel_stats.csv).
# Build here:  bash scripts/exp/topk_scatter_variants.sh build    Run on the GPU box: ... run
set -e
cd "$(dirname "$0")/../.."
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
V="base: m4:-DOMF_FINE_MARGIN=4 m2:-DOMF_FINE_MARGIN=2 u2:-DOMF_FHIST_U=2"
if [ "$1" = build ]; then
  for v in $V; do
    name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
    mkdir -p exp_libs/$name
    for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
      hipcc $F $flags -c omnifed_amd/csrc/$s -o exp_libs/$name/$s.o &
    done
    wait
    hipcc --offload-arch=gfx950 -shared -fPIC -o exp_libs/$name/lib.so exp_libs/$name/*.o
    rm -f exp_libs/$name/*.o
  done
  exit 0
fi
for v in $V; do
  name=${v%%:*}
  OMF_CODEC_LIB_EXPERIMENT=exp_libs/$name/lib.so bash scripts/gpu.sh prof tks_$name --codec topk > /dev/null
done
