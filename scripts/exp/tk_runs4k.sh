#!/bin/bash
# Experiment (GPU box): a larger sample (4 Ki runs per tensor) with one or two sample blocks per
# tensor, against the default (2 Ki runs, one block): Top-K per-kernel times.
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
d=/tmp/omf_sb4096; mkdir -p $d
for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
  timeout -k 10 400 hipcc $F -DOMF_SRUNS_PER_BLOCK=4096 -c omnifed_amd/csrc/$s -o $d/$s.o &
done
wait
timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o $d/lib.so $d/*.o || exit 1
run() {  # name, env...
  local o=gpurun_out/tk4k_$1; shift; rm -rf $o
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- \
      python3 bench.py --codec topk --no-cpu-baseline --no-extras --steps 20 > $o.log 2>&1 || exit 3
}
for rep in 1 2; do
  run base_$rep OMF_TOPK_SAMPLE_RUNS=2048
  run r4k_2blk_$rep OMF_TOPK_SAMPLE_RUNS=4096
  run r4k_1blk_$rep OMF_TOPK_SAMPLE_RUNS=4096 OMF_CODEC_LIB_EXPERIMENT=$d/lib.so
done
