#!/bin/bash
# Experiment (GPU box): fallback counts of the Top-K fast path for fine-bin margins 8 and 2.
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
for m in ${MARGINS:-8 2}; do
  d=/tmp/omf_m$m; mkdir -p $d
  for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
    timeout -k 10 400 hipcc $F -DOMF_FINE_MARGIN=$m -c omnifed_amd/csrc/$s -o $d/$s.o &
  done
  wait
  timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o $d/lib.so $d/*.o || exit 1
  OMF_TOPK_DBG=4 OMF_CODEC_LIB_EXPERIMENT=$d/lib.so timeout -k 10 400 python3 -u scripts/exp/topk_flags2.py ${SEEDS:-3} > gpurun_out/tkf_$m.out 2> gpurun_out/tkf_$m.err || exit 2
  echo "margin $m: calls $(grep -c 'omf_topk: redo' gpurun_out/tkf_$m.err), fallbacks $(grep 'omf_topk: redo' gpurun_out/tkf_$m.err | grep -vc 'redo 0 overflow 0')"
done
