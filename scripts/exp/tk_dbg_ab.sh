#!/bin/bash
# Experiment (GPU box): an OMF_EXPERIMENTS build of the codec library in /tmp, then the Top-K encode
# timed with the output-changing debug switches (OMF_TOPK_DBG: 1 = no bucket ordering, 2 = no
# residual zeroing in the bucket sort), to attribute the bucket sort's time.
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -DOMF_EXPERIMENTS"
mkdir -p /tmp/omf_exp
for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
  timeout -k 10 400 hipcc $F -c omnifed_amd/csrc/$s -o /tmp/omf_exp/$s.o &
done
wait
timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o /tmp/omf_exp/lib.so /tmp/omf_exp/*.o || exit 1
echo built
OMF_CODEC_LIB_EXPERIMENT=/tmp/omf_exp/lib.so timeout -k 10 400 python -u scripts/exp/tk_env_ab.py OMF_TOPK_DBG=0,1,2,3 7
