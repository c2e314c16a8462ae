#!/bin/bash
# Experiment (GPU box): the Top-K threshold margin (OMF_THR_Z sigma + OMF_THR_C samples above the
# expected k*S/n; default 6 sigma + 32).  A narrower margin leaves fewer candidates for the
# fine histogram, scatter and sort, and sends more calls to the exact redo.  Per variant: the
# Top-K GPU tests (on the narrowest), the redo/overflow flags over 48 calls (topk_flags.py,
# OMF_TOPK_DBG=4), and the encode time (tk_runs_sweep.py at 2 Ki runs) interleaved with the
# in-tree build.
set -o pipefail
cd "$(dirname "$0")/../.." && export TMPDIR=/tmp
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude"
build() {
  local d=/tmp/omf_thr_$1; shift; mkdir -p $d
  for s in omf_runtime.cpp omf_qsgd.hip omf_qsgd_ring.hip omf_qsgd_pack.hip omf_topk.hip; do
    (timeout -k 10 400 hipcc $F "$@" -c omnifed_amd/csrc/$s -o $d/$s.o && echo "$d $s" >> gpurun_out/thr_progress.txt) &
  done
  wait
  timeout -k 10 200 hipcc --offload-arch=gfx950 -shared -fPIC -o $d/lib.so $d/*.o || exit 1
}
build z5 -DOMF_THR_Z=5.0 -DOMF_THR_C=16.0
build z4 -DOMF_THR_Z=4.0 -DOMF_THR_C=16.0
build z3 -DOMF_THR_Z=3.0 -DOMF_THR_C=8.0
echo built
OMF_CODEC_LIB_EXPERIMENT=/tmp/omf_thr_z3/lib.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu -k "topk or top_k" tests/ > gpurun_out/thr_check.log 2>&1 || { tail -30 gpurun_out/thr_check.log; exit 4; }
tail -1 gpurun_out/thr_check.log
lib() { [ "$1" = base ] && echo "" || echo /tmp/omf_thr_$1/lib.so; }
for v in base z5 z4 z3; do
  OMF_CODEC_LIB_EXPERIMENT=$(lib $v) OMF_TOPK_DBG=4 timeout -k 10 300 python3 -u scripts/exp/topk_flags.py 12 \
      > gpurun_out/thr_flags_$v.log 2>&1 || exit 5
  echo "$v: $(grep -c 'omf_topk: redo' gpurun_out/thr_flags_$v.log) calls, $(grep 'omf_topk: redo' gpurun_out/thr_flags_$v.log | grep -vc 'redo 0 overflow 0') fell back"
done
for rep in 1 2; do
  for v in base z5 z4 z3; do
    OMF_CODEC_LIB_EXPERIMENT=$(lib $v) timeout -k 10 300 python3 -u scripts/exp/tk_runs_sweep.py 2048 > gpurun_out/thr_${v}_$rep.log 2>&1 || exit 6
    echo "$v $rep $(tail -1 gpurun_out/thr_${v}_$rep.log)"
  done
done
