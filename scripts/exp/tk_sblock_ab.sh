#!/bin/bash
# Experiment (GPU box): Top-K per-kernel times against the sampled runs per sample block (512:
# 4 blocks for a 2 Ki-run tensor, each flushing its LDS histogram with global atomics; 1024, 2048).
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
for m in 512 1024 2048; do
  d=/tmp/omf_sb$m; mkdir -p $d
  for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
    timeout -k 10 400 hipcc $F -DOMF_SRUNS_PER_BLOCK=$m -c omnifed_amd/csrc/$s -o $d/$s.o &
  done
  wait
  timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o $d/lib.so $d/*.o || exit 1
done
echo built
for rep in 1 2; do
for m in 512 1024 2048; do
  o=gpurun_out/tksb_${m}_$rep; rm -rf $o
  OMF_CODEC_LIB_EXPERIMENT=/tmp/omf_sb$m/lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- \
      python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > $o.log 2>&1 || exit 3
done
done
