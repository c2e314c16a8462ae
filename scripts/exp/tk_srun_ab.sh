#!/bin/bash
# Experiment (GPU box): the Top-K sample's run length and count.  A run is kSRun consecutive
# elements read as float4s; the sample kernel's time follows the number of random lines one CU
# has in flight, so 32-element runs (one 128-byte line) at 1 Ki runs per tensor keep the 32 Ki
# samples of the default (16-element runs, 2 Ki per tensor) with half the lines.  Variant r32 is
# built aside (OMF_SRUN=32, 1 Ki runs per block); the Top-K GPU tests run on it first; then
# scripts/exp/tk_runs_sweep.py (Llama-400M encode, medians) alternates the in-tree build and r32.
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
d=/tmp/omf_srun_r32; mkdir -p $d
for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
  (timeout -k 10 400 hipcc $F -DOMF_SRUN=32 -DOMF_SRUNS_PER_BLOCK=1024 -c omnifed_amd/csrc/$s -o $d/$s.o && echo "built $s" >> gpurun_out/srun_progress.txt) &
done
wait
timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o $d/lib.so $d/*.o || exit 1
echo built
OMF_CODEC_LIB_EXPERIMENT=$d/lib.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu -k "topk or top_k" tests/ > gpurun_out/srun_check.log 2>&1 \
    || { tail -30 gpurun_out/srun_check.log; exit 4; }
tail -1 gpurun_out/srun_check.log
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/exp/tk_runs_sweep.py 2048 1024 1536 > gpurun_out/srun_base_$rep.log 2>&1 || exit 5
  tail -1 gpurun_out/srun_base_$rep.log
  OMF_CODEC_LIB_EXPERIMENT=$d/lib.so timeout -k 10 300 python3 -u scripts/exp/tk_runs_sweep.py 1024 512 768 > gpurun_out/srun_r32_$rep.log 2>&1 || exit 6
  tail -1 gpurun_out/srun_r32_$rep.log
done
